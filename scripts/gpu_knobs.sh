#!/bin/bash
# Slab-pass thread-count / fused-phase variants (filter-only bench).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-knobs}
mkdir -p $O
B="python3 bench.py --filter-only --steps 30 --warmup 3 --no-cpu-baseline"
for v in "768 2" "512 2" "768 3" "768 0" "512 0"; do
  set -- $v
  TEXBIAS_CT_NT=$1 TEXBIAS_CT_FUSE=$2 timeout -k 10 300 $B > $O/k_$1_$2.json 2> $O/k_$1_$2.err || { echo "bench $v failed"; tail -20 $O/k_$1_$2.err; exit 1; }
  echo "nt=$1 fuse=$2"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['filter_ms_per_step'], {k:(v['avg_ms'],v.get('GB_s')) for k,v in d['filter_passes'].items()})" $O/k_$1_$2.json
done
echo done
