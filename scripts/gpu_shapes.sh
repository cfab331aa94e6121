#!/bin/bash
# The reference drivers' own training shape (2 x C x 128 x 128 x 64), eager and as a captured HIP graph:
# the C3 chain + U-Net step (--shape 128,128,64 --pad-to 64) and the gibbs-layer driver, JSON lines and a
# steady-state kernel breakdown of each graph run.  Usage (GPU box): TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-shapes}
O=gpurun_out/$T; mkdir -p $O
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 30 --warmup 5 "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  cut -c1-260 $O/$n.json
}
run unet_small --shape 128,128,64 --pad-to 64
run unet_small_graph --shape 128,128,64 --pad-to 64 --graph
run gibbs_layer --model gibbs-layer
run gibbs_layer_graph --model gibbs-layer --graph
for n in unet_small_graph gibbs_layer_graph gibbs_layer; do
  args="--shape 128,128,64 --pad-to 64 --graph"; mk="--marker k_band_fwd"
  [ $n = gibbs_layer_graph ] && args="--model gibbs-layer --graph" && mk="--marker k_slab_fwd --per-step 3"
  [ $n = gibbs_layer ] && args="--model gibbs-layer" && mk="--marker k_slab_fwd --per-step 3"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$n -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 $args > $O/prof_$n.json 2> $O/prof_$n.err || { echo "prof $n failed"; tail -5 $O/prof_$n.err; exit 1; }
  f=$(find $O/prof_$n -name '*kernel_trace.csv' | head -1)
  python3 scripts/steady_stats.py $f --steps 20 $mk --top 40 > $O/steady_$n.txt && head -12 $O/steady_$n.txt
  rm -f $f
done
echo done
