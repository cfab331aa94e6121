cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc
mkdir -p $OUT
B="python3 bench.py --filter-only --steps 30 --warmup 3 --no-cpu-baseline"
R="--kernel-include-regex k_slab|k_kspace|k_salt|k_minmax"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.json 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE $R --output-format csv -d $OUT/fetch -o run -- $B > /dev/null 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE $R --output-format csv -d $OUT/write -o run -- $B > /dev/null 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SALU $R --output-format csv -d $OUT/insts -o run -- $B > /dev/null 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY $R --output-format csv -d $OUT/stall -o run -- $B > /dev/null 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES $R --output-format csv -d $OUT/grbm -o run -- $B > /dev/null 2>&1 || exit 1
echo pmc done
