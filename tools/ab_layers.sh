#!/bin/bash
# A/B per-layer profile in one process pool: tools/ab_layers.sh TAG "ENV_A" "ENV_B" (e.g. FR_AB=no_trans)
T=$1; A=$2; B=$3
for r in 1 2; do
  env $A tools/gpu_layer_profile.sh ${T}a$r > gpurun_out/${T}a$r.txt || exit 1
  env $B tools/gpu_layer_profile.sh ${T}b$r > gpurun_out/${T}b$r.txt || exit 1
done
for f in a1 b1 a2 b2; do echo "$f $(sed -n 3,4p gpurun_out/${T}$f.txt | tr -s ' ' | cut -d' ' -f1,2,8,9 | tr '\n' ' ') $(tail -1 gpurun_out/${T}$f.txt)"; done
