#!/bin/bash
# A/B of match_x3 variants (tools/build_variant.sh): x3 parity tests per variant, then interleaved match_bench
set -o pipefail
O=gpurun_out/x3ab; mkdir -p $O
V=${1:-"base x3rowmajor"}
for v in $V; do
  L=""; [ "$v" != base ] && L=facerecognition_amd/lib/variants/libfrhip_$v.so
  if [ "$v" = base ]; then T="tests/test_gpu_ops.py tests/test_gpu_distributed.py tests/test_gpu_host_api.py"; K=""; else T=tests/test_gpu_ops.py; K=x3; fi
  FR_LIBFRHIP=$L timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $T ${K:+-k $K} > $O/t_$v.log 2>&1 || { echo "$v tests failed"; tail -30 $O/t_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/t_$v.log)"
done
for r in 1 2 3; do
  for v in $V; do
    L=""; [ "$v" != base ] && L=facerecognition_amd/lib/variants/libfrhip_$v.so
    FR_LIBFRHIP=$L timeout -k 10 200 python tools/match_bench.py --iters 50 > $O/b_${v}_$r.log 2>&1 || { echo "$v bench failed"; tail -20 $O/b_${v}_$r.log; exit 1; }
    true
  done
done
