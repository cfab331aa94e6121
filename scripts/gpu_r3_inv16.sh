#!/bin/bash
# Round 3: split-f16 pass C' -- band tests, new tests, every GPU test, then per-pass timing with the
# f16 synthesis on and off (C3, C2).  Usage (GPU box, repo root): bash scripts/gpu_r3_inv16.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3i}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_band.py > $O/tests_band.log 2>&1
rc=$?; grep -cE "PASSED" $O/tests_band.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" $O/tests_band.log | head -30; tail -30 $O/tests_band.log; exit $rc; }
for cfg in c3 c2; do
  for v in 1 0; do
    TEXBIAS_INV16=$v timeout -k 10 200 python -u scripts/pass_bench.py --config $cfg --iters 40 --tag inv16_$v > $O/pass_${cfg}_$v.json 2> $O/pass_${cfg}_$v.err || { echo pass $cfg $v failed; tail -5 $O/pass_${cfg}_$v.err; exit 1; }
    cat $O/pass_${cfg}_$v.json
  done
done
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c4_extremes.py tests/test_gpu_prep.py tests/test_gpu_train_prod.py tests/test_gpu_ops.py tests/test_gpu_zf.py > $O/tests_new.log 2>&1
rc=$?; grep -E "PASSED|FAILED|loss texbias" $O/tests_new.log | tail -40; [ $rc = 0 ] || { tail -60 $O/tests_new.log; exit $rc; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests_all.log 2>&1
rc=$?; tail -3 $O/tests_all.log; [ $rc = 0 ] || { tail -60 $O/tests_all.log; exit $rc; }
echo done
