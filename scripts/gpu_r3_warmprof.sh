#!/bin/bash
# Round 3: Python-level profile of bench.py's first (warmup) step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3d}; mkdir -p $O
timeout -k 10 400 python3 -u -m cProfile -o $O/warm.prof bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/warm.json 2> $O/warm.err || { echo failed; tail -5 $O/warm.err; exit 1; }
python3 - $O/warm.prof > $O/warm_stats.txt <<'PY'
import pstats, sys
s = pstats.Stats(sys.argv[1]); s.sort_stats("cumulative").print_stats(45)
s.sort_stats("tottime").print_stats(25)
PY
grep -E "warmup step" $O/warm.err; echo done
