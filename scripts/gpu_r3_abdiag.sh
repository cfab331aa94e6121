#!/bin/bash
# Round 3: pass_bench for each (variant, TEXBIAS_BAND_DIAG mask) pair.  Usage: TAG "variants" "masks" [c3|c2]
# ("default" = the in-tree library; masked runs are stage attribution only, results invalid by design)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3abd}; mkdir -p $O
for v in $2; do
  for m in $3; do
    if [ $v = default ]; then unset TEXBIAS_LIB; else export TEXBIAS_LIB=var/$v.so; fi
    TEXBIAS_BAND_DIAG=$m timeout -k 10 300 python3 scripts/pass_bench.py --config ${4:-c3} --iters 30 --flush-mb 0 --tag $v > $O/ab_${v}_$m.txt 2>&1 || { tail -5 $O/ab_${v}_$m.txt; exit 1; }
    python3 -c "
import json; l=json.loads(open('$O/ab_${v}_$m.txt').read().strip().splitlines()[-1])
print('$v $m', {k: l[k]['us'] for k in ('forward','kspace','inverse','salt_pepper') if k in l})"
  done
done
echo done
