#!/bin/bash
# Round 3: pass_bench of C3 with the in-tree library and each listed variant (var/NAME.so).  Usage: TAG "names" [tests]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3ab}; mkdir -p $O
if [ -n "$3" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $3 > $O/tests.log 2>&1
  rc=$?; tail -2 $O/tests.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -30 | cut -c1-300; exit $rc; }
fi
for v in default $2 default; do
  if [ $v = default ]; then unset TEXBIAS_LIB; else export TEXBIAS_LIB=var/$v.so; fi
  timeout -k 10 300 python3 scripts/pass_bench.py --config c3 --iters 30 --flush-mb 0 --tag $v > $O/ab_$v.txt 2>&1 || { tail -5 $O/ab_$v.txt; exit 1; }
  python3 -c "
import json; l=json.loads(open('$O/ab_$v.txt').read().strip().splitlines()[-1])
print('$v', {k: l[k]['us'] for k in ('forward','kspace','inverse','salt_pepper') if k in l})"
done
echo done
