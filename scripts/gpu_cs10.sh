cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/cs10; mkdir -p $O
timeout -k 10 300 env TEXBIAS_FWD16_DX_ADD=0 python3 -u bench.py --no-cpu-baseline > $O/bench_noadd.json 2> $O/bench_noadd.err || { echo noadd failed; tail -5 $O/bench_noadd.err; exit 1; }
cut -c1-200 $O/bench_noadd.json
bash scripts/gpu_convstep.sh cs10
