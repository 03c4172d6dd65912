#!/bin/bash
# GPU check on the box: tools/gpu_check.sh TAG [pytest -k expr | all | none] [extra bench args...]
#   tests (all, a -k selection, or none) -> gpurun_out/TAG/tests.log; then bench.py -> gpurun_out/TAG/bench.json
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
T=${1:?tag}; K=${2:-all}; shift 2
O=gpurun_out/$T; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; tail -30 $O/$name.log; exit $rc; fi; }
if [ "$K" = all ]; then
  step tests 600 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread
  grep -E "passed|failed" $O/tests.log | tail -2
elif [ "$K" != none ]; then
  step tests 600 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K"
  grep -E "passed|failed" $O/tests.log | tail -2
fi
step bench 400 python bench.py "$@"
grep '^{' $O/bench.log | tail -1 > $O/bench.json
python tools/show_bench.py $O/bench.json
echo "[$(date +%T)] done"
