#!/bin/bash
# stage13 pre-barrier epilogue: stage tests (bit-identity vs the 14-fragment kernel), same-box A/B
set -o pipefail
O=gpurun_out/r03s5; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_stage.py -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
AB_CLASSES="stage layer3" bash tools/ab.sh "base pre0 pre1p2 pre2" 3 --no-cpu-baseline --no-pmc --steps 20 --warmup 5
