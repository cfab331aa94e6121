#!/bin/bash
# Small and layer-driver shapes (one JSON per line kept): gibbs-layer at the drivers' crop 2x1x128x128x64
# eager / HIP graph, at BraTS size 240x240x160; the C3 chain + U-Net step at the crop 128x128x64 eager / graph;
# and the full-route gibbs-aug chain filter-only at C3.  Usage (GPU box): TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-shapes6}; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['unit'], d['ms_per_step'], {k:(v['kernel'], v['avg_ms'], v.get('GB_s')) for k,v in d['filter_passes'].items()}, d['roofline']['frac'])"; }
run gibbs_layer --model gibbs-layer --steps 20 --warmup 5
run gibbs_layer_graph --model gibbs-layer --steps 20 --warmup 5 --graph
run gibbs_layer_240 --model gibbs-layer --shape 240,240,160 --steps 10 --warmup 3
run unet_small --shape 128,128,64 --pad-to 64 --steps 20 --warmup 5
run unet_small_graph --shape 128,128,64 --pad-to 64 --steps 20 --warmup 5 --graph
run gibbs_aug --filter-only --chain gibbs-aug --steps 20 --warmup 3
run wrap --filter-only --chain wrap --steps 20 --warmup 3
run planes --filter-only --chain planes --steps 20 --warmup 3
echo done
