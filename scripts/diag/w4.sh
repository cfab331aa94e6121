set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/w4; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wrap.py -m gpu > $O/tests.log 2>&1; tail -3 $O/tests.log
timeout -k 10 300 python bench.py --filter-only --chain wrap --steps 20 --warmup 3 > $O/f_wrap.json 2> $O/f_wrap.err; python3 -c "
import json; l=json.loads(open('$O/f_wrap.json').read().strip().splitlines()[-1])
print('wrap', l['filter_ms_per_step'], {k:(v['kernel'],v['avg_ms'],v.get('GB_s')) for k,v in l['filter_passes'].items()})"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/pmc1 -o run -- python3 bench.py --filter-only --chain wrap --steps 4 --warmup 2 --no-cpu-baseline > /dev/null 2> $O/pmc1.err || echo pmc1 failed
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/pmc2 -o run -- python3 bench.py --filter-only --chain wrap --steps 4 --warmup 2 --no-cpu-baseline > /dev/null 2> $O/pmc2.err || echo pmc2 failed
python3 scripts/pmc_summary.py $O/pmc1 $O/pmc2 > $O/pmc_summary.txt 2>&1; grep -A17 "^k_wrap" $O/pmc_summary.txt
timeout -k 10 400 python -u scripts/diag/grad_noise.py > $O/grad_noise.txt 2>&1; grep -A40 "ONE texbias" $O/grad_noise.txt
echo done
