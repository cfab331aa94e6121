#!/bin/bash
# PMC passes on the band kernels (bench.py --filter-only).  Usage: bash scripts/gpu_r2_pmc_inv.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r2q}; O=gpurun_out/$T; mkdir -p $O
F="python3 bench.py --filter-only --steps 10 --warmup 2 --no-cpu-baseline"
R="--kernel-include-regex k_band"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $F > /dev/null 2> $O/trace.err || { echo trace failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU $R --output-format csv -d $O/sq1 -o run -- $F > /dev/null 2> $O/sq1.err || { echo pmc sq1 failed; tail -3 $O/sq1.err; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU $R --output-format csv -d $O/sq2 -o run -- $F > /dev/null 2> $O/sq2.err || { echo pmc sq2 failed; tail -3 $O/sq2.err; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT $R --output-format csv -d $O/gr -o run -- $F > /dev/null 2> $O/gr.err || { echo pmc gr failed; tail -3 $O/gr.err; }
python3 scripts/pmc_summary.py $O/sq1 $O/sq2 $O/gr > $O/pmc_summary.txt 2>&1
cat $O/pmc_summary.txt
grep -h "k_band" $O/trace/*kernel_stats.csv
