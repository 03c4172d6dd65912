#!/bin/bash
# stage13 split fragment (26 + 26 MFMAs per K-step): bit-identity/stage tests, whole-step A/B (no events)
set -o pipefail
O=gpurun_out/r03s17; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_stage.py -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2 3; do
  for v in base nosplit rs3; do
    L=""; [ $v != base ] && L=facerecognition_amd/lib/variants/libfrhip_$v.so
    FR_LIBFRHIP=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-prof --steps 30 --warmup 5 > $O/${v}_$r.log 2>&1 || { echo "$v failed"; tail -20 $O/${v}_$r.log; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/${v}_$r.log $v
  done
done
AB_CLASSES="stage layer3" bash tools/ab.sh "base nosplit" 1 --no-cpu-baseline --no-pmc --steps 20 --warmup 5
