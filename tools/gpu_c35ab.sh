# chain35 (IRV1 repeat_1) check: its parity tests, then same-box IRV1 bench A/B in-tree vs variant builds.
#   tools/gpu_c35ab.sh "variant1 variant2 ..."
set -o pipefail
O=gpurun_out/c35ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -k "chain35" -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed|rel" $O/tests.log | tail -8
for r in 1 2; do
for v in base $1; do
  if [ $v = base ]; then L=""; else L="FR_LIBFRHIP=facerecognition_amd/lib/variants/libfrhip_$v.so"; fi
  env $L timeout -k 10 200 python bench.py --arch irv1_facenet --no-cpu-baseline --no-pmc --no-n1-1m --steps 20 --warmup 5 > $O/${v}_$r.log 2>&1 || { tail -20 $O/${v}_$r.log; exit 1; }
  grep '^{' $O/${v}_$r.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d['kernels']
print('$v', d['value'], 'chain35', k.get('chain block35',{}).get('ms_per_step'))"
done
done
