#!/bin/bash
# Slab-pass diagnostic: time passes A/C with their HBM loads and/or stores skipped (TEXBIAS_DIAG).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-diag}
mkdir -p $O
B="python3 bench.py --filter-only --steps 30 --warmup 3 --no-cpu-baseline"
for d in 0 1 2 3; do
  TEXBIAS_DIAG=$d timeout -k 10 300 $B > $O/d$d.json 2> $O/d$d.err || { echo "bench diag=$d failed"; tail -20 $O/d$d.err; exit 1; }
  echo "diag=$d"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k:v['avg_ms'] for k,v in d['filter_passes'].items()})" $O/d$d.json
done
for nt in 512; do
  TEXBIAS_CT_NT=$nt TEXBIAS_DIAG=3 timeout -k 10 300 $B > $O/n$nt.json 2> $O/n$nt.err || exit 1
  echo "nt=$nt diag=3"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k:v['avg_ms'] for k,v in d['filter_passes'].items()})" $O/n$nt.json
done
echo done
