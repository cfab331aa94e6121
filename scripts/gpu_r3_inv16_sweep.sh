#!/bin/bash
# Round 3: pass C' (k_band_inv16) attribution -- library variants (waves/SIMD, LDS slots) and
# TEXBIAS_BAND_DIAG stage masks under scripts/pass_bench.py (C3 and C2).  Usage: bash scripts/gpu_r3_inv16_sweep.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3s}
mkdir -p $O
run() {  # name cfg env...
  local nm=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 120 python -u scripts/pass_bench.py --config $cfg --iters 40 --tag $nm > $O/$nm.$cfg.json 2> $O/$nm.$cfg.err || { echo "$nm $cfg failed"; tail -3 $O/$nm.$cfg.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/$nm.$cfg.json')); print('$nm', '$cfg', {k: d[k]['us'] for k in ('forward','kspace','inverse','salt_pepper') if k in d})"
}
for cfg in c3 c2; do
  run base $cfg TEXBIAS_BAND_DIAG=0
  for v in inv16_w5s2 inv16_w6s2 inv16_w6s1; do run $v $cfg TEXBIAS_LIB=$GRAFT_REPO_ROOT/var/$v.so; done
  for m in 0x400 0x800 0x1000 0x1800 0x1c00 0x2000 0x4000; do run diag$m $cfg TEXBIAS_BAND_DIAG=$m; done
done
echo done
