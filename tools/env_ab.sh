#!/bin/bash
# Interleaved A/B of environment switches on bench.py's per-kernel event timing:
#   tools/env_ab.sh "base FR_AB=img56" [rounds]     (each item: VAR=value, e.g. FR_AB=no_trans,no_wring, or "base")
set -o pipefail
V=${1:?settings}; N=${2:-2}
O=gpurun_out/env_ab; mkdir -p $O
for r in $(seq 1 $N); do
  for v in $V; do
    tag=$(echo "$v" | tr "=,;/." "_____")
    if [ "$v" = base ]; then env_set=""; else env_set="${v//;/ }"; fi  # several VAR=value: separated by ;
    env $env_set timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-n1-1m --steps 20 --warmup 5 $AB_ARGS > $O/${tag}_$r.log 2>&1 || { echo "$v failed"; tail -20 $O/${tag}_$r.log; exit 1; }
    python - $O/${tag}_$r.log "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = d.get("kernels", {})
print(f"{sys.argv[2]:18s} {d['value']:9.1f} faces/s {d['ms_per_step']:.3f} ms | " +
      " ".join(f"{k}={v['ms_per_step']}" for k, v in list(ks.items())[:8]), flush=True)
PY
  done
done
