set -o pipefail
mkdir -p gpurun_out/r03h
FR_LIBFRHIP=facerecognition_amd/lib/variants/libfrhip_trace.so timeout -k 10 200 python tools/stage_trace.py > gpurun_out/r03h/trace.txt 2>&1 && cat gpurun_out/r03h/trace.txt | tail -12 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc > gpurun_out/r03h/bench.log 2>&1 && grep '^{' gpurun_out/r03h/bench.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms/step', d['ms_per_step'], 'fwd', d.get('forward'))
for k,v in d.get('kernels',{}).items(): print(f'  {k:28s} {v[\"ms_per_step\"]:7.4f} ms  mfma {v[\"mfma_frac\"]:.3f} hbm {v[\"hbm_frac\"]:.3f}')"
