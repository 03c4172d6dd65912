#!/bin/bash
# opt-in branch streams: model tests (incl. replay == eager with FR_BRANCH_STREAMS=1)
set -o pipefail
O=gpurun_out/r03s19; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_models.py -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
