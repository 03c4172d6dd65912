#!/bin/bash
# Timing-experiment builds of libfrhip.so with conv_img.hip compiled under -DFR_IMG_EXP=N
# (1: no weight stream, 2: no patch stream, 4: neither; DMA counts change, so results are garbage
# and the vmcnt waits over-wait) into facerecognition_amd/lib/exp/img$N/.
set -e
cd "$(dirname "$0")/../facerecognition_amd/csrc"
make -s
for n in 1 2 4; do
  d=../lib/exp/img$n; mkdir -p $d build/imgexp$n
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -DFR_IMG_EXP=$n \
    -c conv_img.hip -o build/imgexp$n/conv_img.o
  objs=$(ls build/*.o | grep -v conv_img.o)
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $d/libfrhip.so $objs build/imgexp$n/conv_img.o
done
