# fp8 stage: parity tests, then fp8 and bf16 bench lines
set -o pipefail
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_fp8.py -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $O/fp8.log 2>&1 || { tail -60 $O/fp8.log; exit 1; }
grep -E "rel err|1-cos|agreement|PASS|FAIL|passed|failed" $O/fp8.log | tail -40
for dt in fp8 bf16; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc --dtype $dt > $O/bench_$dt.log 2>&1 || { tail -20 $O/bench_$dt.log; exit 1; }
grep '^{' $O/bench_$dt.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$dt value', d['value'], 'ms/step', d['ms_per_step'], 'fwd', d.get('forward'))
for k,v in d.get('kernels',{}).items(): print(f'  {k:28s} {v[\"ms_per_step\"]:7.4f} ms  mfma {v[\"mfma_frac\"]:.3f} hbm {v[\"hbm_frac\"]:.3f}')"
done
