#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/exp2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_norm.py -x -v --timeout 120 --timeout-method thread > $O/pytest_norm.log 2>&1 || { echo norm tests failed; tail -30 $O/pytest_norm.log; exit 1; }
tail -2 $O/pytest_norm.log
B="python3 bench.py --filter-only --steps 30 --warmup 3 --no-cpu-baseline"
for nt in 512 1024; do
  TEXBIAS_SLAB_NT=$nt timeout -k 10 300 $B > $O/bench_nt$nt.json 2> $O/bench_nt$nt.err || { echo "bench nt=$nt failed"; tail -20 $O/bench_nt$nt.err; exit 1; }
done
timeout -k 10 600 python3 bench.py --no-cpu-baseline > $O/bench_full.json 2> $O/bench_full.err || { echo full bench failed; tail -20 $O/bench_full.err; exit 1; }
cat $O/bench_full.json
R="--kernel-include-regex k_slab|k_kspace|k_salt"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE $R --output-format csv -d $O/fetch -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE $R --output-format csv -d $O/write -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SALU $R --output-format csv -d $O/insts -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY $R --output-format csv -d $O/stall -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS $R --output-format csv -d $O/busy -o run -- $B > /dev/null 2>&1 || exit 1
echo done
