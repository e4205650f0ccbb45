#!/bin/bash
# Link an A/B variant of libmvpose.so: the in-tree objects with one source file replaced.
#   bash tools/build_variant.sh OUT.so csrc_name.hip VARIANT_SOURCE [extra hipcc flags...]
# (run `make` first; the variant source is compiled with the library's flags)
set -e
OUT=$1; NAME=$2; SRC=$3; shift 3
P=multi-camera_3d_pose_estimation_amd
mkdir -p /tmp/variant
cp "$SRC" $P/csrc/.variant_$NAME
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I include -I $P/csrc \
    -munsafe-fp-atomics "$@" -c -x hip $P/csrc/.variant_$NAME -o /tmp/variant/${NAME%.hip}.o
rm -f $P/csrc/.variant_$NAME
OBJS=$(ls $P/build/*.o | grep -v "/${NAME%.hip}.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $P/mvpose/$OUT $OBJS /tmp/variant/${NAME%.hip}.o
echo "built $P/mvpose/$OUT"
