#!/bin/bash
# Round 3: first-step time with MIOpen's naive solvers out of Find; cold then warm find-db.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3e}; mkdir -p $O gpurun_out/miopen2
export TEXBIAS_MIOPEN_DIR=$GRAFT_REPO_ROOT/gpurun_out/miopen2
for run in 1 2; do
  timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$run.json 2> $O/bench_$run.err || { echo "bench $run failed"; tail -5 $O/bench_$run.err; exit 1; }
  grep "warmup step" $O/bench_$run.err; cut -c1-200 $O/bench_$run.json
done
echo done
