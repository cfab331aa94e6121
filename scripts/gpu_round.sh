#!/bin/bash
# One GPU-box session: gpu parity tests, smoke, bench line, rocprofv3 kernel-trace summary.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r1}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo pytest failed; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { echo prof failed; tail -30 $O/prof_bench.err; exit 1; }
echo done
