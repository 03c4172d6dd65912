# 64 / 32-row igemm tiles: bit-exactness tests, then IRV1 and ResNet-50 bench lines (tuner picks)
set -o pipefail
O=gpurun_out/${1:-r06j}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "tile64" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for arch in irv1_facenet resnet50_arcface; do
  timeout -k 10 300 python bench.py --arch $arch --no-cpu-baseline --no-pmc --steps 30 > $O/bench_$arch.log 2>&1 || { tail -20 $O/bench_$arch.log; exit 1; }
  grep '^{' $O/bench_$arch.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$arch value', d['value'], 'ms/step', d['ms_per_step'])
for k,v in sorted(d.get('kernels',{}).items(), key=lambda kv: -kv[1]['ms_per_step'])[:10]: print(f'  {k:28s} {v[\"ms_per_step\"]:7.4f} ms  mfma {v[\"mfma_frac\"]:.3f}')"
done
