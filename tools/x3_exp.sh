#!/bin/bash
# Timing-experiment builds of libfrhip.so with match_x3.hip compiled under -DFR_X3_EXP=N
# (1: no MFMA, 2: no gallery stream, 3: no filter/insert) into facerecognition_amd/lib/exp/N/.
# Run one with FR_LIBFRHIP=facerecognition_amd/lib/exp/N/libfrhip.so python tools/match_bench.py
set -e
cd "$(dirname "$0")/../facerecognition_amd/csrc"
make -s
for n in 1 2 3; do
  d=../lib/exp/$n; mkdir -p $d build/exp$n
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -DFR_X3_EXP=$n \
    -c match_x3.hip -o build/exp$n/match_x3.o
  objs=$(ls build/*.o | grep -v match_x3.o)
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $d/libfrhip.so $objs build/exp$n/match_x3.o
done
