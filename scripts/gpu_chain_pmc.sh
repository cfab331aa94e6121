#!/bin/bash
# Per chain mode: filter-only bench line + rocprofv3 kernel stats, two SQ counter passes and the
# FETCH_SIZE / WRITE_SIZE passes (traffic_<chain>.json).  Usage (GPU box): TAG CHAIN [CHAIN ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift; mkdir -p $O
B="bench.py --filter-only --steps 5 --warmup 2 --no-cpu-baseline"
for ch in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$ch -o run -- python3 bench.py --filter-only --chain $ch --steps 20 --warmup 3 --no-cpu-baseline > $O/filter_$ch.json 2> $O/filter_$ch.err || { echo "$ch stats failed"; tail -5 $O/filter_$ch.err; exit 1; }
  f=$(find $O/prof_$ch -name '*kernel_trace.csv' | head -1); rm -f $f
  cp $(find $O/prof_$ch -name '*kernel_stats.csv' | head -1) $O/kernel_stats_$ch.csv
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
             "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_${ch}_$i -o run -- python3 $B --chain $ch > /dev/null 2> $O/pmc_${ch}_$i.err || { echo "pmc $ch $i failed"; tail -3 $O/pmc_${ch}_$i.err; exit 1; }
  done
  python3 scripts/make_traffic.py $O/pmc_${ch}_3 $O/pmc_${ch}_4 $O/filter_$ch.json $O/traffic_$ch.json "--filter-only --chain $ch --steps 5 --warmup 2" > /dev/null || exit 1
  python3 scripts/pmc_summary.py $O/pmc_${ch}_1 $O/pmc_${ch}_2 > $O/pmc_summary_$ch.txt
  python3 -c "
import json; l=json.loads(open('$O/filter_$ch.json').read().strip().splitlines()[-1])
print('$ch', l['value'], l['filter_ms_per_step'], {k:(v['kernel'],v['avg_ms'],v.get('GB_s')) for k,v in l['filter_passes'].items()})"
done
echo done
