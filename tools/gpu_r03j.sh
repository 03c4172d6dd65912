set -o pipefail
mkdir -p gpurun_out/r03j
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "narrow or every_tile or conv_parity" > gpurun_out/r03j/t.log 2>&1 || { tail -40 gpurun_out/r03j/t.log; exit 1; }
tail -2 gpurun_out/r03j/t.log
bash tools/gpu_layer_profile.sh irv1j --arch irv1_facenet > gpurun_out/r03j/lp.txt 2>&1; head -32 gpurun_out/lp_irv1j/summary.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc --arch irv1_facenet > gpurun_out/r03j/bench_irv1.log 2>&1 && grep '^{' gpurun_out/r03j/bench_irv1.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print('irv1 value', d['value'], 'ms/step', d['ms_per_step'], 'fwd', d.get('forward'))"
bash tools/pmc_run.sh gpurun_out/r03j/pmc_v0 > gpurun_out/r03j/pmc_v0.log 2>&1 && python tools/pmc_summary.py gpurun_out/r03j/pmc_v0 stage > gpurun_out/r03j/pmc_v0.txt && \
FR_STAGE_VARIANT=1 bash tools/pmc_run.sh gpurun_out/r03j/pmc_v1 > gpurun_out/r03j/pmc_v1.log 2>&1 && python tools/pmc_summary.py gpurun_out/r03j/pmc_v1 stage > gpurun_out/r03j/pmc_v1.txt; tail -3 gpurun_out/r03j/pmc_v1.log
