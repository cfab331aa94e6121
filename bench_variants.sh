cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --cudnn-benchmark > gpurun_out/bench_cb.json 2> gpurun_out/bench_cb.err; echo cb rc=$?
