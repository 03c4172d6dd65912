#!/bin/bash
# conv_direct (small-K direct conv): op tests (bit-exact vs igemm tile 0), IRV1 model parity, IRV1 bench A/B
set -o pipefail
O=gpurun_out/r03s7; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread -k "direct" > $O/t_direct.log 2>&1 || { tail -40 $O/t_direct.log; exit 1; }
tail -1 $O/t_direct.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --arch irv1_facenet --steps 20 --warmup 5 > $O/irv1_$r.log 2>&1 || { tail -20 $O/irv1_$r.log; exit 1; }
  tail -1 $O/irv1_$r.log | cut -c1-160
  FR_NO_DIRECT=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --arch irv1_facenet --steps 20 --warmup 5 > $O/irv1_nd_$r.log 2>&1 || { tail -20 $O/irv1_nd_$r.log; exit 1; }
  tail -1 $O/irv1_nd_$r.log | cut -c1-160
done
python tools/show_classes.py $O/irv1_1.log 2>/dev/null | head -30 || true
