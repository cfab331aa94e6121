#!/bin/bash
# Full GPU pass: parity tests, smoke, bench line, rocprofv3 kernel trace + steady-state summary.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --steps 5 > $O/prof_bench.json 2> $O/prof_bench.err || { echo prof failed; tail -30 $O/prof_bench.err; exit 1; }
python3 scripts/steady_stats.py $O/prof/run_kernel_trace.csv --steps 5 --top 30 > $O/steady.txt 2>&1; head -25 $O/steady.txt
echo done
