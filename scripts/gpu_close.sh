#!/bin/bash
# Closing perf record: bench C3 (with CPU baseline), C2, C5; filter-only C3 and C2 + PMC FETCH/WRITE
# passes for roofline.traffic; rocprofv3 kernel trace of the C3 train step (steady-state window) and
# kernel stats of the C2 line.  Usage (GPU box): TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-close}; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 600 python3 -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }; cut -c1-220 $O/$n.json; }
run bench_c3
run bench_c2 --config c2
run bench_c5 --config c5 --no-cpu-baseline
run filter_c3 --filter-only --steps 20 --warmup 3 --no-cpu-baseline
for cfg in c3 c2; do
  A="--config $cfg --filter-only --steps 5 --warmup 2 --no-cpu-baseline"
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$cfg -o run -- python3 bench.py $A > /dev/null 2> $O/pmc_fetch_$cfg.err || { echo fetch $cfg failed; tail -3 $O/pmc_fetch_$cfg.err; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$cfg -o run -- python3 bench.py $A > /dev/null 2> $O/pmc_write_$cfg.err || { echo write $cfg failed; tail -3 $O/pmc_write_$cfg.err; exit 1; }
done
python3 scripts/make_traffic.py $O/pmc_fetch_c3 $O/pmc_write_c3 $O/filter_c3.json $O/traffic_c3.json "--filter-only --steps 5 --warmup 2" > /dev/null || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --config c2 --no-cpu-baseline > $O/prof_c2.json 2> $O/prof_c2.err || { echo prof c2 failed; tail -5 $O/prof_c2.err; exit 1; }
f=$(find $O/prof_c2 -name '*kernel_trace.csv' | head -1); rm -f $f
cp $(find $O/prof_c2 -name '*kernel_stats.csv' | head -1) $O/kernel_stats_c2.csv
python3 scripts/make_traffic.py $O/pmc_fetch_c2 $O/pmc_write_c2 $O/prof_c2.json $O/traffic_c2.json "--config c2 --filter-only --steps 5 --warmup 2" > /dev/null || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_c3.json 2> $O/prof_c3.err || { echo prof failed; tail -5 $O/prof_c3.err; exit 1; }
f=$(find $O/prof_c3 -name '*kernel_trace.csv' | head -1)
python3 scripts/steady_stats.py $f --steps 20 --marker k_band_fwd --top 40 > $O/steady_c3.txt && head -14 $O/steady_c3.txt
rm -f $f
cp $(find $O/prof_c3 -name '*kernel_stats.csv' | head -1) $O/kernel_stats_c3.csv
echo done
