#!/bin/bash
# GPU tests + one default bench line:  tools/gpu_quick_tb.sh TAG
set -o pipefail
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-600
