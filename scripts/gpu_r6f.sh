#!/bin/bash
# A/B on one box: split-f16 A' (TEXBIAS_BAND_FWD16) x C' slot sizing (TEXBIAS_INV16_SLOTS=12: round-5 batches).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r6f}; mkdir -p $O
for rep in 1 2; do
for cfg in "1 0" "0 0" "1 12" "0 12"; do
  set -- $cfg
  TEXBIAS_BAND_FWD16=$1 TEXBIAS_INV16_SLOTS=$2 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b.json 2> $O/b.err || { echo bench failed; tail -5 $O/b.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/b.json')); print('c3 fwd16=$1 slots=$2', d['value'], {k:v['avg_ms'] for k,v in d['filter_passes'].items()}, d['roofline']['frac'])"
  TEXBIAS_BAND_FWD16=$1 TEXBIAS_INV16_SLOTS=$2 timeout -k 10 300 python3 -u bench.py --config c2 --no-cpu-baseline > $O/b.json 2> $O/b.err || { echo c2 failed; tail -5 $O/b.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/b.json')); print('c2 fwd16=$1 slots=$2', d['value'], {k:v['avg_ms'] for k,v in d['filter_passes'].items()}, d['roofline']['frac'])"
done
done
echo done
