#!/bin/bash
# conv_direct with 8-fragment units / no pad below 8 chunks: op tests, IRV1 per-launch profile, IRV1 bench A/B
set -o pipefail
O=gpurun_out/r03s9; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread -k "direct" > $O/t_direct.log 2>&1 || { tail -40 $O/t_direct.log; exit 1; }
tail -1 $O/t_direct.log
bash tools/gpu_layer_profile.sh r03s9_irv1 --arch irv1_facenet > /dev/null || exit 1
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --arch irv1_facenet --steps 20 --warmup 5 > $O/irv1_$r.log 2>&1 || { tail -20 $O/irv1_$r.log; exit 1; }
  tail -1 $O/irv1_$r.log | cut -c1-120
  FR_NO_DIRECT=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --arch irv1_facenet --steps 20 --warmup 5 > $O/irv1_nd_$r.log 2>&1 || { tail -20 $O/irv1_nd_$r.log; exit 1; }
  tail -1 $O/irv1_nd_$r.log | cut -c1-120
done
