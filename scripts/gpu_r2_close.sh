#!/bin/bash
# Round-2 closing measurement, part 1: every GPU test, the C3 bench line (with the CPU baseline),
# the C2 line, rocprofv3 kernel-trace/stats of both.  Usage (GPU box, repo root): bash scripts/gpu_r2_close.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r2g}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 500 python3 -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { echo c3 failed; tail -5 $O/bench_c3.err; exit 1; }
cut -c1-300 $O/bench_c3.json
timeout -k 10 300 python3 -u bench.py --config c2 > $O/bench_c2.json 2> $O/bench_c2.err || { echo c2 failed; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/trace_c3.out 2> $O/trace_c3.err || { echo trace c3 failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c2 -o run -- python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline > $O/trace_c2.out 2> $O/trace_c2.err || { echo trace c2 failed; exit 1; }
echo done
