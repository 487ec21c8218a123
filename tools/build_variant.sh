#!/bin/bash
# Build an A/B variant of the HIP library with extra defines into build/ab_<name>/
# (select it at run time with ANISO_LIB=build/ab_<name>/libaniso_mi355x.so).
# usage: tools/build_variant.sh <name> "-DFOO=1 -DBAR=2"
set -e
NAME=$1
DEFS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/build/ab_$NAME
mkdir -p $D $ROOT/build/include
cp $ROOT/include/*.h $ROOT/build/include/
rm -rf $D/csrc && cp -r $ROOT/aniso_amd/csrc $D/csrc
rm -f $D/csrc/*.o
make -s -C $D/csrc -j8 HIPFLAGS="--offload-arch=gfx950 -munsafe-fp-atomics $DEFS" CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-result $DEFS" 2>&1 | grep -v "warning\|note:\|^ *[0-9]* |\|^ *|\|generated" || true
ls -la $D/libaniso_mi355x.so
