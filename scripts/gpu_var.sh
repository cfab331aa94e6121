#!/bin/bash
# Filter-pass variants by environment (filter-only bench); usage: VARS="ENV=.. ENV=..;ENV=.." gpu_var.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-var}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_k.log 2>&1 || { echo pytest failed; tail -40 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
B="python3 bench.py --filter-only --steps 30 --warmup 3 --no-cpu-baseline"
i=0
IFS=';' read -ra VS <<< "$VARS"
for v in "${VS[@]}"; do
  i=$((i+1))
  env $v timeout -k 10 300 $B > $O/v$i.json 2> $O/v$i.err || { echo "bench $v failed"; tail -20 $O/v$i.err; exit 1; }
  echo "[$v]"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k:v['avg_ms'] for k,v in d['filter_passes'].items()})" $O/v$i.json
done
echo done
