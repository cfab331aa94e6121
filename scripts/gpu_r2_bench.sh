#!/bin/bash
# Round-2 measurement: the default bench line (C3 chain + U-Net train step, CPU baseline in three
# modes), the C2 line (Gibbs truncation alone, 4x128^3), rocprofv3 kernel-trace/stats of both, and
# PMC FETCH/WRITE passes of the filter kernels for roofline.traffic.
# Usage (GPU box, repo root): bash scripts/gpu_r2_bench.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r2b}
O=gpurun_out/$T
mkdir -p $O
R="--kernel-include-regex k_band|k_salt|k_sap|k_slab|k_kspace|k_minmax|k_copy"
timeout -k 10 600 python3 -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { echo bench c3 failed; tail -5 $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
timeout -k 10 300 python3 -u bench.py --config c2 > $O/bench_c2.json 2> $O/bench_c2.err || { echo bench c2 failed; tail -5 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
B3="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o run -- $B3 > $O/trace_c3.out 2> $O/trace_c3.err || { echo trace c3 failed; exit 1; }
B2="python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c2 -o run -- $B2 > $O/trace_c2.out 2> $O/trace_c2.err || { echo trace c2 failed; exit 1; }
F3="python3 bench.py --filter-only --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 200 $F3 > $O/bench_f3.json 2> /dev/null || { echo f3 failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE $R --output-format csv -d $O/fetch_c3 -o run -- $F3 > /dev/null 2>&1 || { echo pmc fetch c3 failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE $R --output-format csv -d $O/write_c3 -o run -- $F3 > /dev/null 2>&1 || { echo pmc write c3 failed; exit 1; }
python3 scripts/make_traffic.py $O/fetch_c3 $O/write_c3 $O/bench_f3.json $O/traffic_c3.json "--filter-only (C3: B=2 x 4 x 240x240x155, padded to 160)" > /dev/null || { echo traffic c3 failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE $R --output-format csv -d $O/fetch_c2 -o run -- $B2 > /dev/null 2>&1 || { echo pmc fetch c2 failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE $R --output-format csv -d $O/write_c2 -o run -- $B2 > /dev/null 2>&1 || { echo pmc write c2 failed; exit 1; }
python3 scripts/make_traffic.py $O/fetch_c2 $O/write_c2 $O/bench_c2.json $O/traffic_c2.json "--config c2 (B=16 x 4 x 128^3)" > /dev/null || { echo traffic c2 failed; exit 1; }
cat $O/traffic_c3.json $O/traffic_c2.json
for t in trace_c3 trace_c2; do echo "== $t"; find $O/$t -name "*kernel_stats.csv" -exec head -25 {} \; ; done
