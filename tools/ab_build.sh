#!/bin/bash
# Build a variant library from gcm.hip at git revision REV into
# boringssl_amd/csrc/build/ab_NAME/libbssl_amd.so (A/B timing on one box:
# BSSL_AMD_LIB selects it).  Usage: tools/ab_build.sh NAME REV [extra hipcc flags]
set -eu
NAME=$1; REV=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/boringssl_amd/csrc
O=$C/build/ab_$NAME
mkdir -p $O
git -C $ROOT show $REV:boringssl_amd/csrc/gcm.hip > $O/gcm.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$ROOT/include -I$C -fvisibility=hidden "$@" -c $O/gcm.hip -o $O/gcm.o
OBJS=$(ls $C/build/*.o | grep -v gcm.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libbssl_amd.so $O/gcm.o $OBJS -Wl,-Bsymbolic
echo $O/libbssl_amd.so
