#!/bin/bash
# Prebuild variant libraries of libmhq_huff.so in this container (parallel):
#   bash tools/abvar.sh OUTDIR name=flags ...
# then time them on the GPU box with tools/ab.sh (VDIR=OUTDIR).
OUT=$1; shift
mkdir -p "$OUT"
SRC=minhq_amd/csrc
build_one() {
  name=${1%%=*}; flags=${1#*=}
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $flags -o "$OUT/lib_$name.so" \
    $SRC/huff_decode.hip $SRC/huff_decode_stream.hip $SRC/read_strings.hip $SRC/huff_encode.hip $SRC/enc_packed.hip $SRC/huff_scan.hip $SRC/str_frame.hip $SRC/huff_table.cpp $SRC/mhq_api.cpp \
    > "$OUT/build_$name.log" 2>&1 && echo "built $name" || { echo "FAILED $name"; tail -5 "$OUT/build_$name.log"; }
}
export -f build_one; export OUT SRC
printf '%s\n' "$@" | xargs -P 4 -I{} bash -c 'build_one "$@"' _ {}
