#!/bin/bash
# Per-layer time for the given igemm tile ids (band on for W=14): tools/tile_sweep2.sh PREFIX id...
P=$1; shift
for t in "$@"; do
  FR_AB=conv_tile=$t tools/gpu_layer_profile.sh ${P}$t > /dev/null || exit 1
  echo "tile $t: $(tail -1 gpurun_out/lp_${P}$t/summary.txt)"
done
