cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu5.log 2>&1; echo pytest rc=$?
for tb in 32768 16384 65536; do
TEXBIAS_TILE_BYTES=$tb timeout -k 10 300 python bench.py --filter-only --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench_filter3_t$tb.json 2> gpurun_out/bench_filter3_t$tb.err || exit 1
done
echo done
