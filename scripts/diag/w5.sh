set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/w5; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wrap.py -m gpu > $O/tests.log 2>&1; tail -2 $O/tests.log
timeout -k 10 300 python bench.py --filter-only --chain wrap --steps 20 --warmup 3 > $O/f_wrap.json 2> $O/f_wrap.err; python3 -c "
import json; l=json.loads(open('$O/f_wrap.json').read().strip().splitlines()[-1])
print('wrap', l['filter_ms_per_step'], {k:(v['kernel'],v['avg_ms'],v.get('GB_s')) for k,v in l['filter_passes'].items()})"
timeout -k 10 400 python -u scripts/diag/adn_check.py > $O/adn.txt 2>&1; grep -v Warning $O/adn.txt | tail -12
timeout -k 10 300 python -u scripts/wgrad_bench.py > $O/wgrad.txt 2>&1; cat $O/wgrad.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/pmc1 -o run -- python3 scripts/wgrad_bench.py > /dev/null 2> $O/pmc1.err || echo pmc1 failed
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/pmc2 -o run -- python3 scripts/wgrad_bench.py > /dev/null 2> $O/pmc2.err || echo pmc2 failed
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc3 -o run -- python3 scripts/wgrad_bench.py > /dev/null 2> $O/pmc3.err || echo pmc3 failed
python3 scripts/pmc_summary.py $O/pmc1 $O/pmc2 $O/pmc3 > $O/pmc_summary.txt 2>&1; grep -A19 "^k_conv3d" $O/pmc_summary.txt | head -100
echo done
