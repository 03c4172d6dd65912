#!/bin/bash
# stage13w (one wave per SIMD, 13 fragments, ring 6): bit-identity test, same-box env A/B
set -o pipefail
O=gpurun_out/r03s10; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_stage.py -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread -k "variants" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
bash tools/env_ab.sh "base FR_STAGE_VARIANT=2" 3
