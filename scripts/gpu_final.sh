#!/bin/bash
# Round close: the whole GPU suite + smoke, then the closing perf record (scripts/gpu_close.sh).  Usage: TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-final}
bash scripts/gpu_suite.sh $T/suite || exit 1
bash scripts/gpu_close.sh $T/close || exit 1
