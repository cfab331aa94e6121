set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/w3; mkdir -p $O
timeout -k 10 300 python -u scripts/diag/grad_noise.py > $O/grad_noise.txt 2>&1; sed -n 3,12p $O/grad_noise.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train_prod.py tests/test_gpu_norm.py -m gpu -s > $O/train_prod.log 2>&1; grep -E "passed|failed|loss texbias|texbias .* aten-f32" $O/train_prod.log | head -12
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/pmc$i -o run -- python3 bench.py --filter-only --chain gibbs-aug --steps 4 --warmup 2 --no-cpu-baseline > $O/pmc$i.out 2> $O/pmc$i.err || { echo "pmc $i failed"; tail -3 $O/pmc$i.err; }
done
python3 scripts/pmc_summary.py $O/pmc1 $O/pmc2 $O/pmc3 $O/pmc4 > $O/pmc_summary.txt 2>&1; head -40 $O/pmc_summary.txt
echo done
