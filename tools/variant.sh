#!/bin/bash
# Same-box A/B builds of one kernel source: tools/variant.sh NAME SRC.hip [extra hipcc flags]
# builds facerecognition_amd/lib/variants/libfrhip_NAME.so = the current library with SRC.hip compiled in place of
# the csrc file of the same base name (load it with FR_LIBFRHIP=<path>; bench.py / tests pick it up).
set -e
N=${1:?name}; SRC=${2:?source}; shift 2
R=$(cd "$(dirname "$0")/.." && pwd); C=$R/facerecognition_amd/csrc
make -C $C -s -j8
base=$(basename $SRC .hip)
mkdir -p $C/build_var $R/facerecognition_amd/lib/variants
cp $SRC $C/build_var/$base.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -I$C "$@" -c $C/build_var/$base.hip -o $C/build_var/$base.o
srcs=$(sed -n 's/^SRCS := //p' $C/Makefile)
objs=""; for f in $srcs; do b=${f%.*}; [ "$b" = "$base" ] || objs="$objs $C/build/$b.o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs $C/build_var/$base.o -o $R/facerecognition_amd/lib/variants/libfrhip_$N.so
echo "built facerecognition_amd/lib/variants/libfrhip_$N.so"
