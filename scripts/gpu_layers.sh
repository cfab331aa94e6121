#!/bin/bash
# The in-model layer drivers (bench.py --model gibbs-layer / spike-layer) at the drivers' 1 x 128 x 128 x 64
# crops and at BraTS size, each with a rocprofv3 kernel-stats summary.  Usage (GPU box): TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-layers}; mkdir -p $O
for m in gibbs-layer spike-layer; do
  for sh in "" "--shape 240,240,160 --batch 2"; do
    tag=$m$([ -n "$sh" ] && echo _brats)
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$tag -o run -- python3 bench.py --model $m $sh --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$tag.json 2> $O/bench_$tag.err || { echo "$tag failed"; tail -5 $O/bench_$tag.err; exit 1; }
    f=$(find $O/prof_$tag -name '*kernel_trace.csv' | head -1); rm -f $f
    cp $(find $O/prof_$tag -name '*kernel_stats.csv' | head -1) $O/kernel_stats_$tag.csv
    cut -c1-230 $O/bench_$tag.json
  done
done
echo done
