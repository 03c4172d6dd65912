# IRV1 parity + speed for FR_AB settings: tools/gpu_irv1par.sh TAG AB...
set -o pipefail
T=${1:?tag}; shift; O=gpurun_out/$T; mkdir -p $O
for ab in "$@"; do
  FR_AB=$ab timeout -k 10 300 python -u -m pytest tests/test_gpu_models.py -x -q -s -p no:cacheprovider --timeout 200 --timeout-method thread -k "irv1_full_batch_bs256 and bf16" > "$O/par_$ab.log" 2>&1 || { tail -30 "$O/par_$ab.log"; exit 1; }
  echo "AB=$ab"; grep -E "vs oracle max|agreement" "$O/par_$ab.log" | head -3
  FR_AB=$ab timeout -k 10 300 python bench.py --arch irv1_facenet --no-cpu-baseline --no-pmc --steps 30 > "$O/bench_$ab.log" 2>&1 || { tail -20 "$O/bench_$ab.log"; exit 1; }
  grep '^{' "$O/bench_$ab.log" | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print('  value', d['value'], 'ms/step', d['ms_per_step'])"
done
