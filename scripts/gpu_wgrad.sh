#!/bin/bash
# GPU check of the conv weight-gradient kernel: its parity tests, then the full bench line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-wg}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -v --timeout 120 --timeout-method thread > $O/pytest_conv.log 2>&1 || { echo conv tests failed; tail -40 $O/pytest_conv.log; exit 1; }
tail -3 $O/pytest_conv.log
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --steps 5 > $O/prof_bench.json 2> $O/prof_bench.err || { echo prof failed; tail -30 $O/prof_bench.err; exit 1; }
echo done
