cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/few1; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv.py > $O/tests.log 2>&1 || { echo tests failed; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for u in 1 2 4; do
  TEXBIAS_CONVT_FEW_UNROLL=$u timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$u -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/b$u.json 2> $O/b$u.err || { echo "u$u failed"; tail -3 $O/b$u.err; exit 1; }
  echo "unroll $u: $(grep convT_fewout $(find $O/p$u -name '*kernel_stats.csv') | cut -d, -f1-5)"
  rm -f $(find $O/p$u -name '*kernel_trace.csv')
done
