#!/bin/bash
# branch-parallel graph capture: replay == eager tests, model parity, IRV1 / R50 no-prof bench A/B
set -o pipefail
O=gpurun_out/r03s18; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_stage.py -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2 3; do
  for arch in irv1_facenet resnet50_arcface; do
    for v in base FR_NO_BRANCH_STREAMS=1; do
      E=""; [ $v != base ] && E=$v
      env $E timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-prof --arch $arch --steps 30 --warmup 5 > $O/${arch}_${v}_$r.log 2>&1 || { echo "$v failed"; tail -20 $O/${arch}_${v}_$r.log; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/${arch}_${v}_$r.log "$arch $v"
    done
  done
done
