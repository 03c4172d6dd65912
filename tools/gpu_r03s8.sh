#!/bin/bash
# IRV1 per-launch profile with and without conv_direct
set -o pipefail
bash tools/gpu_layer_profile.sh r03s8_irv1 --arch irv1_facenet && \
FR_NO_DIRECT=1 bash tools/gpu_layer_profile.sh r03s8_irv1_nd --arch irv1_facenet
