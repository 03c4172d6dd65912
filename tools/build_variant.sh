#!/bin/bash
# Timing-experiment build of libfrhip.so with extra compile flags, beside the product library:
#   tools/build_variant.sh NAME "-DFR_STAGE_SB=0 ..."  ->  facerecognition_amd/lib/variants/libfrhip_NAME.so
# Select it at run time with FR_LIBFRHIP=<path> (facerecognition_amd/_native.py); tools/ab.sh runs A/B.
set -e
N=${1:?name}; F=${2:-}
R=$(cd $(dirname $0)/.. && pwd)
S=${SRC_ROOT:-$R}  # sources from another checkout (e.g. a git worktree of an older commit)
C=$S/facerecognition_amd/csrc
B=$R/facerecognition_amd/csrc/build_$N
mkdir -p $B $R/facerecognition_amd/lib/variants
objs=""
for s in conv_igemm.hip conv_fp8.hip conv_band.hip conv_stage.hip conv_stage8.hip conv_split_stage.hip conv_wring.hip conv_direct.hip conv_small.hip conv_img.hip conv_rows.hip conv_stem.hip misc.hip match.hip match_x3.hip preprocess.hip mtcnn.hip blas.cpp engine.cpp; do
  [ -f $C/$s ] || continue  # an older checkout (SRC_ROOT) may predate a source
  o=$B/${s%.*}.o; objs="$objs $o"
  x=""; [ "${s##*.}" = cpp ] && x="-x hip"
  [ "$s" = conv_rows.hip ] && x="-mllvm -amdgpu-mfma-vgpr-form"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I$S/include $F $x -c $C/$s -o $o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o $R/facerecognition_amd/lib/variants/libfrhip_$N.so -L/opt/rocm/lib -lhipblaslt -Wl,-rpath,/opt/rocm/lib
echo "built facerecognition_amd/lib/variants/libfrhip_$N.so"
