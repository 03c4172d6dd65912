# ResNet-50 stem kernel check: tools/gpu_stemr50.sh TAG [FR_AB settings to compare, default "" no_stem_r50]
set -o pipefail
T=${1:?tag}; shift; O=gpurun_out/$T; mkdir -p $O
ABS=("$@"); [ ${#ABS[@]} -eq 0 ] && ABS=("" "no_stem_r50" "" "no_stem_r50")
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py -k "stem_r50 or bneck28 or chain_r50" -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed|rel|1-cos" $O/tests.log | tail -20
i=0
for ab in "${ABS[@]}"; do
  i=$((i+1))
  FR_AB=$ab timeout -k 10 300 python bench.py --arch resnet50_arcface --no-cpu-baseline --no-pmc --steps 30 > "$O/bench_${i}_$ab.log" 2>&1 || { tail -20 "$O/bench_${i}_$ab.log"; exit 1; }
  grep '^{' "$O/bench_${i}_$ab.log" | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print('AB=$ab value', d['value'], 'ms/step', d['ms_per_step'])
for k,v in sorted(d.get('kernels',{}).items(), key=lambda kv: -kv[1]['ms_per_step'])[:8]: print(f'  {k:28s} {v[\"ms_per_step\"]:7.4f} ms  mfma {v[\"mfma_frac\"]:.3f} hbm {v[\"hbm_frac\"]:.3f}')"
done
