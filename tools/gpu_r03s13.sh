#!/bin/bash
# conv_rows ping-pong variant: rows op tests, model tests, whole-step A/B vs FR_ROWS_PP=0
set -o pipefail
O=gpurun_out/r03s13; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread -k "rows or img56" > $O/t_rows.log 2>&1 || { tail -40 $O/t_rows.log; exit 1; }
tail -1 $O/t_rows.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_stage.py -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2 3; do
  for v in base FR_ROWS_PP=0; do
    E=""; [ $v != base ] && E=$v
    env $E timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-prof --steps 30 --warmup 5 > $O/${v}_$r.log 2>&1 || { echo "$v failed"; tail -20 $O/${v}_$r.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/${v}_$r.log $v
  done
done
bash tools/env_ab.sh "base FR_ROWS_PP=0" 1
