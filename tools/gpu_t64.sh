set -o pipefail
O=gpurun_out/r06i; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "tile64" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
FR_AB=tune_log=1 timeout -k 10 300 python bench.py --arch irv1_facenet --no-cpu-baseline --no-pmc --steps 30 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep "tune M=2304\|tune M=16384" $O/bench.log | head -12
grep '^{' $O/bench.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms/step', d['ms_per_step'])
for k,v in sorted(d.get('kernels',{}).items(), key=lambda kv: -kv[1]['ms_per_step'])[:14]: print(f'  {k:28s} {v[\"ms_per_step\"]:7.4f} ms  mfma {v[\"mfma_frac\"]:.3f}')"
