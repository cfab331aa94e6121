#!/bin/bash
# Round 3 quick loop: band tests, per-pass timing of the split-f16 C' on/off (C3, C2), then any extra
# pytest node ids given.  Usage (GPU box): bash scripts/gpu_r3_quick.sh TAG [pytest node ids...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3q}; shift
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_band.py > $O/tests_band.log 2>&1
rc=$?; grep -cE "PASSED" $O/tests_band.log; [ $rc = 0 ] || { grep -E "Error|assert" $O/tests_band.log | head -30; tail -30 $O/tests_band.log; exit $rc; }
for cfg in c3 c2; do
  for v in 1 0; do
    TEXBIAS_INV16=$v timeout -k 10 200 python -u scripts/pass_bench.py --config $cfg --iters 40 --tag inv16_$v > $O/pass_${cfg}_$v.json 2> $O/pass_${cfg}_$v.err || { echo pass $cfg $v failed; tail -5 $O/pass_${cfg}_$v.err; exit 1; }
    cat $O/pass_${cfg}_$v.json
  done
done
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu "$@" > $O/tests_extra.log 2>&1
  rc=$?; grep -E "PASSED|FAILED|loss texbias|^  model" $O/tests_extra.log | tail -40; [ $rc = 0 ] || { tail -40 $O/tests_extra.log; exit $rc; }
fi
echo done
