#!/bin/bash
# Interleaved A/B of library variants (tools/build_variant.sh) on bench.py's per-kernel event timing:
#   tools/ab.sh "base sb1 sb2" [rounds] [bench args]   ("base" = the product library)
# Prints, per run, the step time and the per-class ms/step of the classes named in AB_CLASSES.
set -o pipefail
V=${1:?variants}; N=${2:-2}; shift 2; ARGS=${*:-"--no-cpu-baseline --steps 20 --warmup 5"}
O=gpurun_out/ab; mkdir -p $O
for r in $(seq 1 $N); do
  for v in $V; do
    L=""; [ "$v" != base ] && L=facerecognition_amd/lib/variants/libfrhip_$v.so
    FR_LIBFRHIP=$L timeout -k 10 200 python bench.py $ARGS > $O/${v}_$r.log 2>&1 || { echo "$v failed"; tail -20 $O/${v}_$r.log; exit 1; }
    python - $O/${v}_$r.log $v "${AB_CLASSES:-stage layer3}" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = d.get("kernels", {})
cls = [c for c in sys.argv[3].split(",")]
print(f"{sys.argv[2]:8s} {d['value']:9.1f} faces/s  {d['ms_per_step']:.3f} ms/step  " +
      "  ".join(f"{c}={ks.get(c, {}).get('ms_per_step')}" for c in cls), flush=True)
PY
  done
done
