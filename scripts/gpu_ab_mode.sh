#!/bin/bash
# A/B of library variants on one filter-only chain (bench.py --filter-only --chain CHAIN), alternating per
# library, twice.  Usage (GPU box): TAG CHAIN LIB...  (LIB relative to the repo, "default" = in-tree build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-abm}; CH=$2; shift 2; mkdir -p $O
for rep in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = default ]; then unset TEXBIAS_LIB; else export TEXBIAS_LIB=$GRAFT_REPO_ROOT/$lib; fi
    timeout -k 10 300 python3 -u bench.py --filter-only --chain $CH --steps 20 --warmup 3 --no-cpu-baseline > $O/b.json 2> $O/b.err || { echo bench failed; tail -5 $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/b.json')); print('$CH $lib', d['ms_per_step'], {k:(v['kernel'],v['avg_ms']) for k,v in d['filter_passes'].items()}, d['roofline']['frac'])"
  done
done
echo done
