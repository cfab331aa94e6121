#!/bin/bash
# c5 (DCGAN) variants: default, channels_last, batch 256.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-c5ab}
mkdir -p gpurun_out/$T
i=0
for v in "" "--channels-last" "--batch 256" "--batch 256 --channels-last"; do
  timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 3 $v > gpurun_out/$T/b_$i.json 2> gpurun_out/$T/b_$i.err || { echo "bench $v failed"; tail -3 gpurun_out/$T/b_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/$T/b_$i.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
  i=$((i+1))
done
