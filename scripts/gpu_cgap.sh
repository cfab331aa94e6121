#!/bin/bash
# Pass C' (k_band_inv16) in the filter-only chain (back to back) vs inside the train-step bench: the
# same counter groups in both contexts.  Usage (GPU box): TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-cgap}; mkdir -p $O
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
           "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_TAG_STALL_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/filt_$i -o run -- python3 bench.py --filter-only --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2> $O/filt_$i.err || { echo "filt $i failed"; tail -3 $O/filt_$i.err; exit 1; }
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d $O/train_$i -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > /dev/null 2> $O/train_$i.err || { echo "train $i failed"; tail -3 $O/train_$i.err; exit 1; }
done
python3 scripts/pmc_summary.py $O/filt_1 $O/filt_2 $O/filt_3 | grep -A22 "^k_band_inv16" > $O/cgap_filter.txt
python3 scripts/pmc_summary.py $O/train_1 $O/train_2 $O/train_3 | grep -A22 "^k_band_inv16" > $O/cgap_train.txt
paste $O/cgap_filter.txt $O/cgap_train.txt
echo done
