#!/bin/bash
# Per-layer time of every igemm tile (band off) and of the default plan: tools/tile_sweep.sh PREFIX
P=${1:-sw}
for t in 0 1 2 3 4 5 6; do
  FR_AB=no_band,conv_tile=$t tools/gpu_layer_profile.sh ${P}$t > /dev/null || exit 1
done
tools/gpu_layer_profile.sh ${P}def > /dev/null || exit 1
echo sweep done
