#!/bin/bash
# Interleaved A/B of library variants (tools/build_variant.sh) on the config-4 shard match (tools/match_bench.py):
#   tools/ab_match.sh "base noseed" [rounds] [match_bench args]   ("base" = the product library)
set -o pipefail
V=${1:?variants}; N=${2:-2}; shift 2; ARGS=${*:-"--only-rows 125000 --iters 30"}
for r in $(seq 1 $N); do
  for v in $V; do
    L=""; [ "$v" != base ] && L=facerecognition_amd/lib/variants/libfrhip_$v.so
    echo -n "$v: "; FR_LIBFRHIP=$L timeout -k 10 120 python tools/match_bench.py $ARGS || { echo "$v failed"; exit 1; }
  done
done
