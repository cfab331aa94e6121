#!/bin/bash
# Pass A 16-B staged loads: parity (kernel tests), then filter-only variants.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-raw16}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_k.log 2>&1 || { echo pytest failed; tail -40 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
B="python3 bench.py --filter-only --steps 30 --warmup 3 --no-cpu-baseline"
for v in "0 x" "1 x" "2 x"; do
  set -- $v
  TEXBIAS_INV_PREF=$1 timeout -k 10 300 $B > $O/r$1_$2.json 2> $O/r$1_$2.err || { echo "bench $v failed"; tail -20 $O/r$1_$2.err; exit 1; }
  echo "invpref=$1"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k:v['avg_ms'] for k,v in d['filter_passes'].items()})" $O/r$1_$2.json
done
echo done
