# quick GPU check: tools/gpu_quick.sh TAG "pytest -k expr" [extra bench args]
set -o pipefail
T=${1:?tag}; K=${2:-}; shift 2
O=gpurun_out/$T; mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc "$@" > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms/step', d['ms_per_step'], 'fwd', d.get('forward'))
for k,v in d.get('kernels',{}).items(): print(f'  {k:28s} {v[\"ms_per_step\"]:7.4f} ms  mfma {v[\"mfma_frac\"]:.3f} hbm {v[\"hbm_frac\"]:.3f}')"
