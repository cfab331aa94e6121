#!/bin/bash
# Filter-pass experiments: workgroup-size variants + PMC counters of the filter kernels.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-fexp}
mkdir -p $O
B="python3 bench.py --filter-only --steps 30 --warmup 3 --no-cpu-baseline"
for nt in 512 1024; do
  TEXBIAS_SLAB_NT=$nt timeout -k 10 300 $B > $O/bench_nt$nt.json 2> $O/bench_nt$nt.err || { echo "bench nt=$nt failed"; tail -20 $O/bench_nt$nt.err; exit 1; }
done
R="--kernel-include-regex k_slab|k_kspace|k_salt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/trace.json 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE $R --output-format csv -d $O/fetch -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE $R --output-format csv -d $O/write -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SALU $R --output-format csv -d $O/insts -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY $R --output-format csv -d $O/stall -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS $R --output-format csv -d $O/busy -o run -- $B > /dev/null 2>&1 || exit 1
echo done
