#!/bin/bash
# Build a variant of libatz_accel.so with extra compile flags, for A/B runs through ATZ_LIB.
# usage: tools/variant.sh <name> <flags...>   -> antiz_amd/_build/libatz_<name>.so
N=$1; shift
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -x hip -Wno-unused-result -Wno-unused-value \
  "$@" antiz_amd/csrc/atz_accel.cpp -o antiz_amd/_build/libatz_$N.so
