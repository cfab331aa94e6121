#!/bin/bash
# Round 3: pass C' prologue attribution (TEXBIAS_BAND_DIAG: 0x2000 prologue only, +0x8000 no table
# loads, +0x10000 no fragment loads, 0x4000 launch only), with and without the cache flush.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3g}
mkdir -p $O
for fl in 1024 0; do
  for m in 0 0x4000 0x2000 0xa000 0x12000 0x1a000; do
    TEXBIAS_BAND_DIAG=$m timeout -k 10 120 python -u scripts/pass_bench.py --config c3 --iters 30 --flush-mb $fl > $O/pro_$m.$fl.json 2> $O/pro_$m.$fl.err || { echo "$m failed"; tail -3 $O/pro_$m.$fl.err; exit 1; }
    python -c "import json; d=json.load(open('$O/pro_$m.$fl.json')); print('flush $fl diag $m', {k: d[k]['us'] for k in ('forward','kspace','inverse','salt_pepper') if k in d})"
  done
done
