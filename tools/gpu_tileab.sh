# New igemm tiles: their bit-exactness tests, then same-box bench A/B (in-tree library vs a variant build) on IRV1,
# ResNet-50 and IResNet100.  tools/gpu_tileab.sh TAG VARIANT
set -o pipefail
T=${1:?tag}; V=${2:?variant}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "tile64 or igemm" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for arch in irv1_facenet irv1_facenet resnet50_arcface iresnet100; do
  for v in base $V; do
    if [ $v = base ]; then L=""; else L="FR_LIBFRHIP=facerecognition_amd/lib/variants/libfrhip_$v.so"; fi
    env $L timeout -k 10 300 python bench.py --arch $arch --no-cpu-baseline --no-pmc --steps 30 > $O/bench_${arch}_$v.log 2>&1 || { tail -20 $O/bench_${arch}_$v.log; exit 1; }
    grep '^{' $O/bench_${arch}_$v.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$arch $v', d['value'], d['ms_per_step'])
for k,v in sorted(d.get('kernels',{}).items(), key=lambda kv: -kv[1]['ms_per_step'])[:8]: print(f'  {k:28s} {v[\"ms_per_step\"]:7.4f} ms x{v[\"launches\"]}')"
  done
done
