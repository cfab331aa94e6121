#!/bin/bash
# fused DU / RE slab phases: parity (both variants) and filter-only timing per TEXBIAS_CT_FUSE
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-fuse}
mkdir -p $O
for f in 3 0; do
  TEXBIAS_CT_FUSE=$f timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $O/pytest_f$f.log 2>&1 || { echo "tests fuse=$f failed"; tail -40 $O/pytest_f$f.log; exit 1; }
  tail -1 $O/pytest_f$f.log
done
for f in 0 1 2 3; do
  TEXBIAS_CT_FUSE=$f timeout -k 10 300 python bench.py --filter-only --steps 30 --warmup 3 --no-cpu-baseline > $O/filter_f$f.json 2> $O/filter_f$f.err || { echo "filter bench fuse=$f failed"; tail -20 $O/filter_f$f.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/filter_f$f.json').read().strip().splitlines()[-1]);print('fuse=$f', d['filter_passes'])"
done
echo done
