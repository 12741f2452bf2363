#!/bin/bash
# Build a variant library from one kernel source (SRC, default gcm.hip) at git
# revision REV (or the working tree: REV=WT) with extra hipcc flags into
# boringssl_amd/csrc/build/ab_NAME/libbssl_amd.so, linked with the current
# objects of every other source (A/B timing on one box: BSSL_AMD_LIB selects
# it).  EXTRA: files copied next to the source first (quoted includes found
# there win: e.g. a regenerated gcm_bs_io.inc).
# Usage: [SRC=chacha.hip] [EXTRA="f ..."] tools/ab_build.sh NAME REV [hipcc flags]
set -eu
NAME=$1; REV=$2; shift 2
SRC=${SRC:-gcm.hip}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/boringssl_amd/csrc
O=$C/build/ab_$NAME
mkdir -p $O
for f in ${EXTRA:-}; do cp "$f" $O/; done
if [ "$REV" = WT ]; then cp $C/$SRC $O/$SRC; else git -C $ROOT show $REV:boringssl_amd/csrc/$SRC > $O/$SRC; fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$ROOT/include -I$C -fvisibility=hidden "$@" -c $O/$SRC -o $O/variant.o
OBJS=$(ls $C/build/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $O/libbssl_amd.so $O/variant.o $OBJS -Wl,-Bsymbolic
echo $O/libbssl_amd.so
