#!/bin/bash
# stage13w ring depth 3 / 6 / 9 vs the 8-wave kernel, whole-step timing without per-kernel events
set -o pipefail
O=gpurun_out/r03s11; mkdir -p $O
for r in 1 2 3; do
  for v in base w6 w3 w9; do
    L=""; E=""
    case $v in w6) E="FR_STAGE_VARIANT=2";; w3) E="FR_STAGE_VARIANT=2"; L=facerecognition_amd/lib/variants/libfrhip_r3.so;; w9) E="FR_STAGE_VARIANT=2"; L=facerecognition_amd/lib/variants/libfrhip_r9.so;; esac
    env $E FR_LIBFRHIP=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-prof --steps 30 --warmup 5 > $O/${v}_$r.log 2>&1 || { echo "$v failed"; tail -20 $O/${v}_$r.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/${v}_$r.log $v
  done
done
