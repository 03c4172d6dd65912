#!/bin/bash
# Timing-only A/B of the layer3 stage kernel switches (FR_STAGE_DBG bits, conv_stage.hip):
#   tools/stage_exp.sh "0 1 2 3"   -> stage ms/step per setting (bench.py per-kernel events)
mkdir -p gpurun_out/stage_exp
for d in ${1:-0 1 2 3}; do
  FR_STAGE_DBG=$d timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/stage_exp/d$d.log 2>&1 || { tail -5 gpurun_out/stage_exp/d$d.log; exit 1; }
  python - $d <<'PY'
import json, sys
j = json.loads(open(f"gpurun_out/stage_exp/d{sys.argv[1]}.log").read().strip().splitlines()[-1])
k = j["kernels"].get("stage layer3", {})
print(f"dbg={sys.argv[1]} stage ms/step={k.get('ms_per_step')} tflops={k.get('tflops')} total ms/step={j['ms_per_step']}")
PY
done
