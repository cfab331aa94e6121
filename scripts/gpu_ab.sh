#!/bin/bash
# A/B of library variants on one box: alternating C3 bench runs (and C2) per library.  Usage: TAG LIB...
# (each LIB a path relative to the repo, "default" = the in-tree libtexbias.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ab}; shift; mkdir -p $O
for rep in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = default ]; then unset TEXBIAS_LIB; else export TEXBIAS_LIB=$GRAFT_REPO_ROOT/$lib; fi
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b.json 2> $O/b.err || { echo bench failed; tail -5 $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/b.json')); print('c3 $lib', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['filter_passes'].items()}, d['roofline']['frac'])"
    timeout -k 10 300 python3 -u bench.py --config c2 --no-cpu-baseline > $O/b.json 2> $O/b.err || { echo c2 failed; tail -5 $O/b.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/b.json')); print('c2 $lib', d['value'], {k:v['avg_ms'] for k,v in d['filter_passes'].items()}, d['roofline']['frac'])"
  done
done
echo done
