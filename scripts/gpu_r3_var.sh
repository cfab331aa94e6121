#!/bin/bash
# Round 3: band tests on the default library, then pass_bench (C3 and C2, no flush) over the default
# library and every var/*.so variant.  Usage (GPU box): bash scripts/gpu_r3_var.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3v}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --tb=short --timeout 200 --timeout-method thread -m gpu tests/test_gpu_band.py > $O/tests_band.log 2>&1
rc=$?; grep -cE "PASSED" $O/tests_band.log; [ $rc = 0 ] || { grep -E "Error|assert" $O/tests_band.log | head -30 | cut -c1-300; exit $rc; }
for cfg in c3 c2; do
  for lib in default var/*.so; do
    nm=$(basename $lib .so)
    if [ $lib = default ]; then unset TEXBIAS_LIB; else export TEXBIAS_LIB=$GRAFT_REPO_ROOT/$lib; fi
    timeout -k 10 120 python -u scripts/pass_bench.py --config $cfg --iters 40 --flush-mb 0 --tag $nm > $O/$nm.$cfg.json 2> $O/$nm.$cfg.err || { echo "$nm $cfg failed"; tail -3 $O/$nm.$cfg.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$nm.$cfg.json')); print('$nm', '$cfg', {k: d[k]['us'] for k in ('forward','kspace','inverse','salt_pepper') if k in d})"
  done
  unset TEXBIAS_LIB
done
echo done
