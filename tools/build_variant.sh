#!/bin/bash
# Build an A/B variant of liblthm_hip.so: one kernel source replaced / recompiled with extra
# flags, linked with the other objects of the normal build (make first).
#   bash tools/build_variant.sh NAME SRC.hip "EXTRA FLAGS"
# -> recommendations_amd/liblthm_hip_NAME.so (select with LTHM_LIB_PATH)
set -e
cd "$(dirname "$0")/.."
NAME=$1; SRC=$2; EXTRA=$3
C=recommendations_amd/csrc
base=$(basename "$SRC" .hip)
base=${base%%_*}   # loss_3loop.hip replaces loss.o
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Werror=shadow -Wno-unused-function -Wno-unused-variable -Wno-unused-result -munsafe-fp-atomics -I$C"
[ "$base" = loss ] && FLAGS="$FLAGS -fno-slp-vectorize"
mkdir -p $C/build/var
/opt/rocm/bin/hipcc $FLAGS $EXTRA -c "$SRC" -o $C/build/var/${base}_$NAME.o
OBJS=$(ls $C/build/*.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS $C/build/var/${base}_$NAME.o -o recommendations_amd/liblthm_hip_$NAME.so
echo "built recommendations_amd/liblthm_hip_$NAME.so"
