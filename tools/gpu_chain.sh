# IRV1 fused-kernel check: tools/gpu_chain.sh TAG [FR_AB settings to compare, default "" no_chain]
set -o pipefail
T=${1:?tag}; shift; O=gpurun_out/$T; mkdir -p $O
ABS=("$@"); [ ${#ABS[@]} -eq 0 ] && ABS=("" "no_chain")
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed|rel|1-cos" $O/tests.log | tail -20
for ab in "${ABS[@]}"; do
  FR_AB=$ab timeout -k 10 300 python bench.py --arch irv1_facenet --no-cpu-baseline --no-pmc --steps 30 > "$O/bench_$ab.log" 2>&1 || { tail -20 "$O/bench_$ab.log"; exit 1; }
  grep '^{' "$O/bench_$ab.log" | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print('AB=$ab value', d['value'], 'ms/step', d['ms_per_step'])
for k,v in sorted(d.get('kernels',{}).items(), key=lambda kv: -kv[1]['ms_per_step'])[:12]: print(f'  {k:28s} {v[\"ms_per_step\"]:7.4f} ms  mfma {v[\"mfma_frac\"]:.3f} hbm {v[\"hbm_frac\"]:.3f}')"
done
