#!/bin/bash
# Round-2 filter-kernel profile: rocprofv3 kernel trace + stats, PMC traffic and SQ counter passes
# of bench.py --filter-only.  Usage: bash scripts/gpu_r2_prof.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r2p}
O=gpurun_out/$T
mkdir -p $O
F="python3 bench.py --filter-only --steps 10 --warmup 2 --no-cpu-baseline"
R="--kernel-include-regex k_band|k_salt|k_slab|k_kspace|k_minmax"
timeout -k 10 300 $F > $O/bench_filter.json 2> $O/bench_filter.err || { echo bench failed; exit 1; }
cat $O/bench_filter.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $F > /dev/null 2> $O/trace.err || { echo trace failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE $R --output-format csv -d $O/fetch -o run -- $F > /dev/null 2>&1 || { echo pmc fetch failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE $R --output-format csv -d $O/write -o run -- $F > /dev/null 2>&1 || { echo pmc write failed; exit 1; }
python3 scripts/make_traffic.py $O/fetch $O/write $O/bench_filter.json $O/traffic.json > /dev/null || { echo traffic failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS $R --output-format csv -d $O/sq1 -o run -- $F > /dev/null 2> $O/sq1.err || { echo pmc sq1 failed; tail -3 $O/sq1.err; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD $R --output-format csv -d $O/sq2 -o run -- $F > /dev/null 2> $O/sq2.err || { echo pmc sq2 failed; tail -3 $O/sq2.err; }
python3 scripts/pmc_summary.py $O/sq1 $O/sq2 $O/fetch $O/write > $O/pmc_summary.txt 2>&1
cat $O/traffic.json
cat $O/pmc_summary.txt
grep -h "k_band\|k_salt" $O/trace/*kernel_stats.csv 2>/dev/null || find $O/trace -name "*stats*"
