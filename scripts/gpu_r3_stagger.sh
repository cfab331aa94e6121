#!/bin/bash
# Round 3: pass_bench of C3 for a list of C' stagger values (TEXBIAS_INV16_STAGGER).  Usage: TAG "v v ..."
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3s}; mkdir -p $O
for v in $2; do
  TEXBIAS_INV16_STAGGER=$v timeout -k 10 300 python3 scripts/pass_bench.py --config c3 --iters 30 --flush-mb 0 > $O/stag_$v.txt 2>&1 || { tail -5 $O/stag_$v.txt; exit 1; }
  python3 -c "
import json; l=json.loads(open('$O/stag_$v.txt').read().strip().splitlines()[-1])
print('stagger $v', {k: l[k]['us'] for k in ('forward','kspace','inverse','salt_pepper') if k in l})"
done
echo done
