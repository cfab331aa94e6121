#!/bin/bash
# SQ counters of the 16-channel conv (scripts/diag/x3_bench.py: 13 calls of tb_conv3d_fwd16 at the C3 shape)
# and of the weight gradients (scripts/wgrad_bench.py), one counter group per pass.  Usage: TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-cpmc}; mkdir -p $O
i=0
B=${2:-scripts/diag/x3_bench.py}
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/pmc$i -o run -- python3 $B > $O/pmc$i.out 2> $O/pmc$i.err || { echo "pmc $i failed"; tail -3 $O/pmc$i.err; }
done
python3 scripts/pmc_summary.py $O/pmc1 $O/pmc2 $O/pmc3 > $O/summary.txt; grep -E -A20 "^k_conv" $O/summary.txt | head -120
echo done
