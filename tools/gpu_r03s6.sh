#!/bin/bash
# raw v_min_f32 in the stage epilogues (no canonicalize): stage tests, same-box A/B vs HEAD and with PRIO=2
set -o pipefail
O=gpurun_out/r03s6; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_stage.py tests/test_gpu_fp8.py -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
AB_CLASSES="stage layer3,stage layer2,stage layer1" bash tools/ab.sh "base head p2" 3 --no-cpu-baseline --no-pmc --steps 20 --warmup 5
