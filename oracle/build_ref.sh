#!/usr/bin/env bash
# Build the REAL reference (jagannatharjun/AntiZ v0) from its own sources where they lie
# under /root/reference, into oracle/_ref/ (git-ignored, but it travels to the GPU box).
#
#   oracle/_ref/uncomp        reference CLI: main.cpp + vendored zlib 1.2.8 + TCLAP
#   oracle/_ref/libz128.so    the vendored zlib 1.2.8 as a shared library
#   oracle/_ref/libzref.so    oracle/zref_shim.c (ours) linked on the vendored zlib: main.cpp's call sequences
#
# Nothing from /root/reference is copied: sources are compiled in place; the only adapter is a
# symlink that resolves main.cpp's `#include "AtzData.h"` to the real ATZData.h (case mismatch,
# main.cpp:1).  `-include cstring` supplies memcpy for main.cpp:959,967 (g++ 11 no longer pulls it
# in transitively).  This is test infrastructure only: the product never links or executes it.
set -euo pipefail
REF=/root/reference
HERE="$(cd "$(dirname "$0")" && pwd)"
OUT="$HERE/_ref"
if [ ! -d "$REF" ]; then
  echo "build_ref: $REF absent (GPU box): using prebuilt $OUT" >&2
  exit 0
fi
Z="$REF/includes, tools, stuff/zlib test/zlib128"
T="$REF/includes, tools, stuff/tclap/tclap-1.2.1/include"
mkdir -p "$OUT/obj" "$OUT/inc"
ln -sf "$REF/ATZData.h" "$OUT/inc/AtzData.h"
objs=()
for f in adler32 compress crc32 deflate infback inffast inflate inftrees trees uncompr zutil; do
  o="$OUT/obj/$f.o"
  if [ ! -f "$o" ] || [ "$Z/$f.c" -nt "$o" ]; then
    gcc -O3 -fPIC -c "$Z/$f.c" -o "$o"
  fi
  objs+=("$o")
done
gcc -shared -o "$OUT/libz128.so" "${objs[@]}"
ar rcs "$OUT/libz128.a" "${objs[@]}"
gcc -O2 -fPIC -shared -I"$Z" "$HERE/zref_shim.c" "$OUT/libz128.a" -Wl,-Bsymbolic -Wl,--exclude-libs,ALL -o "$OUT/libzref.so"
if [ ! -f "$OUT/uncomp" ] || [ "$REF/main.cpp" -nt "$OUT/uncomp" ]; then
  g++ -O3 -std=c++14 -DHAVE_LONG_LONG -include cstring -I"$OUT/inc" -I"$Z" -I"$T" \
      "$REF/main.cpp" "$OUT/libz128.a" -o "$OUT/uncomp"
fi
echo "build_ref: ok -> $OUT"
