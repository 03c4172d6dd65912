# Fused-kernel epilogue change check: chain / stem tests, then IRV1 and ResNet-50 bench lines.  tools/gpu_relu_ab.sh TAG
set -o pipefail
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_chain.py -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for a in irv1_facenet resnet50_arcface; do
  timeout -k 10 300 python bench.py --arch $a --no-cpu-baseline --no-pmc --steps 30 > $O/bench_$a.log 2>&1 || { tail -20 $O/bench_$a.log; exit 1; }
  grep '^{' $O/bench_$a.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$a', d['value'], 'ms/step', d['ms_per_step'])
for k,v in sorted(d.get('kernels',{}).items(), key=lambda kv: -kv[1]['ms_per_step'])[:8]: print(f'  {k:28s} {v[\"ms_per_step\"]:7.4f} ms')"
done
