#!/bin/bash
# Build diagnostic variants of libmhq_huff.so into $1 (run on the GPU box or here).
OUT=${1:-/tmp/mhq_variants}; shift
mkdir -p "$OUT"
SRC=minhq_amd/csrc
for v in "$@"; do
  name=${v%%=*}; flags=${v#*=}
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $flags -o "$OUT/lib_$name.so" \
    $SRC/huff_decode.hip $SRC/huff_encode.hip $SRC/huff_scan.hip $SRC/str_frame.hip $SRC/huff_table.cpp $SRC/mhq_api.cpp || exit 1
done
