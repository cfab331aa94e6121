#!/bin/bash
# Tuning pass: conv parity tests, wgrad / channel-sum microbench variants, PMC counters of the
# filter passes, full bench line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-tune}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_norm.py -x -q --timeout 120 --timeout-method thread > $O/pytest_conv.log 2>&1 || { echo conv tests failed; tail -40 $O/pytest_conv.log; exit 1; }
tail -2 $O/pytest_conv.log
for yb in 8 4 2 1; do
  TAG=yb$yb TEXBIAS_WGRAD_YB=$yb timeout -k 10 200 python scripts/wgrad_bench.py >> $O/wgrad.txt 2>&1 || { echo wgrad bench failed; tail -20 $O/wgrad.txt; exit 1; }
done
for nb in 256 1024; do
  TAG=nb$nb TEXBIAS_WGRAD_BLOCKS=$nb timeout -k 10 200 python scripts/wgrad_bench.py >> $O/wgrad.txt 2>&1 || { echo wgrad bench failed; tail -20 $O/wgrad.txt; exit 1; }
done
cat $O/wgrad.txt
B="python3 bench.py --filter-only --steps 20 --warmup 3 --no-cpu-baseline"
R="--kernel-include-regex k_slab|k_kspace"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES $R --output-format csv -d $O/insts -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE $R --output-format csv -d $O/stall -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE $R --output-format csv -d $O/fetch -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE $R --output-format csv -d $O/write -o run -- $B > /dev/null 2>&1 || exit 1
python3 scripts/pmc_summary.py $O > $O/pmc_summary.txt 2>&1; cat $O/pmc_summary.txt
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
echo done
