#!/bin/bash
# Build an alternate libdasa_hip (diagnosis A/B) from the release objects with ONE source recompiled under
# extra flags:  tools/build_variant.sh <name> <source.hip> <extra hipcc flags...>
#   -> dasa_amd/build/variant_<name>/libdasa_hip.so ; load it with DASA_LIB=<that path>
set -e
NAME=$1; SRC=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=$ROOT/dasa_amd/build
OUT=$ROOT/dasa_amd/variant_$NAME
mkdir -p $OUT
FLAGS="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-pass-failed -Wno-inline-asm -fno-slp-vectorize -fno-vectorize -Xclang -target-feature -Xclang -packed-fp32-ops -I$ROOT/include"
/opt/rocm/bin/hipcc $FLAGS "$@" -c $ROOT/dasa_amd/csrc/$SRC -o $OUT/$SRC.o
OBJS=""
for o in $B/*.hip.o; do
  [ "$(basename $o)" = "$SRC.o" ] && continue
  OBJS="$OBJS $o"
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/libdasa_hip.so $OBJS $OUT/$SRC.o
echo $OUT/libdasa_hip.so
