#!/bin/bash
# Round 3: pass_bench of C3 under a list of TEXBIAS_BAND_DIAG masks (C' stage attribution; results of
# a masked run are invalid by design).  Usage (GPU box): TAG "mask mask ..." [tests]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3d}; mkdir -p $O
if [ -n "$3" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $3 > $O/tests.log 2>&1
  rc=$?; tail -2 $O/tests.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -30 | cut -c1-300; exit $rc; }
fi
for m in $2; do
  TEXBIAS_BAND_DIAG=$m timeout -k 10 300 python3 scripts/pass_bench.py --config c3 --iters 30 --flush-mb 0 > $O/pass_$m.txt 2>&1 || { tail -5 $O/pass_$m.txt; exit 1; }
  python3 -c "
import json; l=json.loads(open('$O/pass_$m.txt').read().strip().splitlines()[-1])
print('$m', {k: l[k]['us'] for k in ('forward','kspace','inverse','salt_pepper') if k in l})"
done
echo done
