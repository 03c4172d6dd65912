#!/bin/bash
# stage13 loop-head drain fix: GPU tests, bench, same-box A/B against the unfixed build
set -o pipefail
O=gpurun_out/r03s2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
AB_CLASSES="stage layer3,stage layer2" bash tools/ab.sh "base nofix" 3 --no-cpu-baseline --no-pmc --steps 20 --warmup 5
