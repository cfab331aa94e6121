cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "p0 TEXBIAS_CONV16_PERSIST=0" "p1 TEXBIAS_CONV16_PERSIST=1" "p0b TEXBIAS_CONV16_PERSIST=0" "p1b TEXBIAS_CONV16_PERSIST=1"; do set -- $v; t=$1; shift; timeout -k 10 200 env TAG=$t "$@" python3 scripts/diag/conv_kern_bench.py 2>&1 | grep fwd16 || exit 1; done
bash scripts/gpu_convstep.sh cs8
