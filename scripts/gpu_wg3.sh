#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-wg3}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_loss.py -x -q --timeout 120 --timeout-method thread > $O/pytest_conv.log 2>&1 || { echo conv tests failed; tail -40 $O/pytest_conv.log; exit 1; }
tail -2 $O/pytest_conv.log
TAG=wg3 timeout -k 10 200 python scripts/wgrad_bench.py > $O/wgrad.txt 2>&1 || { echo wgrad bench failed; tail -20 $O/wgrad.txt; exit 1; }
grep -v amdgpu.ids $O/wgrad.txt
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
echo done
