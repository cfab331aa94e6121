#!/bin/bash
# Train-step A/B of library variants on one box: rocprofv3 kernel stats of the C3 bench per library (the
# kernels whose names match PATTERN printed with their per-call averages), then scripts/gpu_ab.sh.
# Usage (GPU box): [BENCH_ARGS="..."] TAG PATTERN LIB...   (LIB relative to the repo, "default" = the in-tree
# build; BENCH_ARGS replaces the C3 defaults of the profiled runs, and then the gpu_ab.sh lines are skipped)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-stepab}; PAT=$2; shift 2; O=gpurun_out/$T; mkdir -p $O
for L in "$@"; do
  if [ "$L" = default ]; then unset TEXBIAS_LIB; else export TEXBIAS_LIB=$GRAFT_REPO_ROOT/$L; fi
  N=$(basename $L)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$N -o run -- python3 bench.py ${BENCH_ARGS:---steps 5 --warmup 2} --no-cpu-baseline > $O/b_$N.json 2> $O/p_$N.err || { echo "prof $L failed"; tail -3 $O/p_$N.err; exit 1; }
  rm -f $(find $O/p_$N -name '*kernel_trace.csv')
  python3 -c "
import csv, glob, re
f = glob.glob('$O/p_$N/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if re.search(r'$PAT', r['Name']): print('$N', r['Name'][:90], r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
import json
d = json.loads(open('$O/b_$N.json').read().strip().splitlines()[-1]); print('$N', 'value', d['value'], 'ms/step', d['ms_per_step'])"
done
unset TEXBIAS_LIB
if [ -z "$BENCH_ARGS" ]; then bash scripts/gpu_ab.sh $T "$@"; fi
