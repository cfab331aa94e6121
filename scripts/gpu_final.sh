#!/bin/bash
# Round measurement: GPU parity tests, smoke, PMC traffic of the filter passes, bench line,
# rocprofv3 kernel-trace summary of the bench.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-final}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
F="python3 bench.py --filter-only --steps 10 --warmup 2 --no-cpu-baseline"
R="--kernel-include-regex k_slab|k_kspace"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE $R --output-format csv -d $O/fetch -o run -- $F > /dev/null 2>&1 || { echo pmc fetch failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE $R --output-format csv -d $O/write -o run -- $F > /dev/null 2>&1 || { echo pmc write failed; exit 1; }
python3 scripts/make_traffic.py $O/fetch $O/write $O/traffic.json > /dev/null && cp $O/traffic.json profiles/r1d/traffic.json || { echo traffic failed; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --steps 5 > $O/prof_bench.json 2> $O/prof_bench.err || { echo prof failed; tail -30 $O/prof_bench.err; exit 1; }
python3 scripts/steady_stats.py $O/prof/run_kernel_trace.csv --steps 5 --top 30 > $O/steady.txt 2>&1; head -12 $O/steady.txt
echo done
