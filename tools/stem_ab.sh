#!/bin/bash
# A/B of the persistent fused stem (default) against one block per tile (FR_STEM_PERSIST=0):
# u8-path model tests first, then alternating bench runs; prints the stem kernel time of each.
set -o pipefail
O=gpurun_out/stem_ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_host_api.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for p in 1 0; do
    FR_STEM_PERSIST=$p timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b${p}_$i.log 2>&1 || { tail -20 $O/b${p}_$i.log; exit 1; }
    python -c "import json;d=json.loads(open('$O/b${p}_$i.log').read().strip().splitlines()[-1]);print('persist=$p',d['value'],d['kernels']['stem u8 fused'])"
  done
done
