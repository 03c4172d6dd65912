#!/bin/bash
# SQ counters of match_x3 variants at 2048 x 125k: tools/gpu_x3pmc.sh TAG "name1 name2 ..." (base = in-tree library)
set -o pipefail
T=${1:?tag}; V=${2:?variants}
for v in $V; do
  if [ "$v" = base ]; then unset FR_LIBFRHIP; else export FR_LIBFRHIP=$(pwd)/facerecognition_amd/lib/variants/libfrhip_$v.so; fi
  tools/pmc_match.sh gpurun_out/$T/$v --only-rows 125000 --iters 5 || exit 1
  python tools/pmc_summary.py gpurun_out/$T/$v match_x3 > gpurun_out/$T/$v.txt 2>&1
  echo "== $v"; cat gpurun_out/$T/$v.txt
done
