set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/cgpmc; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_gemm.py tests/test_gpu_norm.py > $O/tests.log 2>&1; echo tests rc $?
for L in "conv 256 256 15 15 10 1 3" "conv 16 32 120 120 80 2 3"; do
  n=$(echo $L | tr ' ' '_')
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/p1_$n -o run -- python3 scripts/diag/cg_one.py $L > $O/p1_$n.log 2>&1 || { echo pmc1 $n failed; tail -3 $O/p1_$n.log; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/p2_$n -o run -- python3 scripts/diag/cg_one.py $L > $O/p2_$n.log 2>&1 || { echo pmc2 $n failed; tail -3 $O/p2_$n.log; exit 1; }
  timeout -s KILL 60 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$n -o run -- python3 scripts/diag/cg_one.py $L > $O/kt_$n.log 2>&1 || { echo kt $n failed; exit 1; }
done
echo done
