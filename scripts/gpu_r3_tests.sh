#!/bin/bash
# Round 3: the listed GPU test files first (new ones), then (optionally) every GPU test.
# Usage (GPU box, repo root): bash scripts/gpu_r3_tests.sh TAG "tests/a.py tests/b.py" [all]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3t}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu $2 > $O/tests_new.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|loss texbias" $O/tests_new.log | tail -40; [ $rc = 0 ] || { tail -60 $O/tests_new.log; exit $rc; }
if [ "$3" = all ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests_all.log 2>&1
  rc=$?; tail -3 $O/tests_all.log; [ $rc = 0 ] || { tail -60 $O/tests_all.log; exit $rc; }
fi
echo done
