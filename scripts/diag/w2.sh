set -o pipefail
O=gpurun_out/w2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wrap.py tests/test_gpu_kernels.py tests/test_gpu_band.py tests/test_gpu_point.py tests/test_gpu_ops.py -m gpu > $O/tests.log 2>&1; tail -3 $O/tests.log
for ch in wrap gibbs-aug; do
  timeout -k 10 300 python bench.py --filter-only --chain $ch --steps 20 --warmup 3 > $O/f_$ch.json 2> $O/f_$ch.err; python3 -c "
import json; l=json.loads(open('$O/f_$ch.json').read().strip().splitlines()[-1])
print('$ch', l['filter_ms_per_step'], {k:(v['kernel'],v['avg_ms'],v.get('GB_s')) for k,v in l['filter_passes'].items()})"
done
TEXBIAS_KSPACE_PERSIST=0 timeout -k 10 300 python bench.py --filter-only --chain gibbs-aug --steps 20 --warmup 3 > $O/f_gibbs_np.json 2> $O/f_gibbs_np.err; python3 -c "
import json; l=json.loads(open('$O/f_gibbs_np.json').read().strip().splitlines()[-1])
print('gibbs nopersist', l['filter_ms_per_step'], {k:(v['kernel'],v['avg_ms'],v.get('GB_s')) for k,v in l['filter_passes'].items()})"
timeout -k 10 300 python -u scripts/diag/grad_noise.py > $O/grad_noise.txt 2>&1; head -12 $O/grad_noise.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train_prod.py -m gpu -k matches_aten -s > $O/train_prod.log 2>&1; grep -E "passed|failed|loss texbias|texbias .* aten-f32" $O/train_prod.log | head -12
