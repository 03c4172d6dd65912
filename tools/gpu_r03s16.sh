#!/bin/bash
# conv_direct 1x1 kernel (operand B from global): op tests, op sweep, IRV1 bench A/B and per-launch profile
set -o pipefail
O=gpurun_out/r03s16; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread -k "direct" > $O/t_direct.log 2>&1 || { tail -40 $O/t_direct.log; exit 1; }
tail -1 $O/t_direct.log
bash tools/gpu_r03s16_sweep.sh | tail -24 || exit 1
bash tools/gpu_layer_profile.sh r03s16_irv1 --arch irv1_facenet > /dev/null || exit 1
for r in 1 2; do
  for v in base FR_NO_DIRECT=1; do
    E=""; [ $v != base ] && E=$v
    env $E timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-prof --arch irv1_facenet --steps 30 --warmup 5 > $O/${v}_$r.log 2>&1 || { echo "$v failed"; tail -20 $O/${v}_$r.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/${v}_$r.log $v
  done
done
