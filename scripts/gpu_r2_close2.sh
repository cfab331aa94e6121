#!/bin/bash
# Round-2 closing measurement, part 2: PMC FETCH_SIZE / WRITE_SIZE passes of the filter kernels
# (C3 filter-only, C2) for roofline.traffic, and the C5 (DCGAN) bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r2g}
mkdir -p $O
R="--kernel-include-regex k_band|k_salt|k_sap|k_slab|k_kspace|k_minmax|k_copy"
F3="python3 bench.py --filter-only --steps 10 --warmup 2 --no-cpu-baseline"
B2="python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 200 $F3 > $O/bench_f3.json 2> /dev/null || { echo f3 failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE $R --output-format csv -d $O/fetch_c3 -o run -- $F3 > /dev/null 2>&1 || { echo pmc fetch c3 failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE $R --output-format csv -d $O/write_c3 -o run -- $F3 > /dev/null 2>&1 || { echo pmc write c3 failed; exit 1; }
python3 scripts/make_traffic.py $O/fetch_c3 $O/write_c3 $O/bench_f3.json $O/traffic_c3.json "--filter-only (C3: B=2 x 4 x 240x240x155, padded to 160)" > /dev/null || { echo traffic c3 failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE $R --output-format csv -d $O/fetch_c2 -o run -- $B2 > /dev/null 2>&1 || { echo pmc fetch c2 failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE $R --output-format csv -d $O/write_c2 -o run -- $B2 > /dev/null 2>&1 || { echo pmc write c2 failed; exit 1; }
timeout -k 10 200 $B2 > $O/bench_c2_short.json 2> /dev/null || { echo c2 short failed; exit 1; }
python3 scripts/make_traffic.py $O/fetch_c2 $O/write_c2 $O/bench_c2_short.json $O/traffic_c2.json "--config c2 (B=16 x 4 x 128^3)" > /dev/null || { echo traffic c2 failed; exit 1; }
cat $O/traffic_c3.json
timeout -k 10 400 python3 -u bench.py --config c5 > $O/bench_c5.json 2> $O/bench_c5.err || { echo c5 failed; exit 1; }
cut -c1-300 $O/bench_c5.json
