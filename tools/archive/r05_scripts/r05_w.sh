#!/bin/bash
# Round 5 call w: decode groups on one window read (MHQ_DEC_TRIPLE) and the group length with pairs, A/B.
set -o pipefail
OUT=${1:-gpurun_out/r05w}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel decode --configs northstar,config2,config3,config2print \
  --libs base=minhq_amd/libmhq_huff.so,triple=build/v/lib_triple.so,pair4=build/v/lib_pair4.so,pair2=build/v/lib_pair2.so \
  --check triple,pair4,pair2 > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v "amdgpu.ids\|check" "$OUT/ab.txt"
