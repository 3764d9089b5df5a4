#!/bin/bash
# Round 5 call u: decode fast loop with two steps per window read (MHQ_DEC_PAIR) A/B.
set -o pipefail
OUT=${1:-gpurun_out/r05u}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel decode --configs northstar,config2,config3,config2print \
  --libs base=minhq_amd/libmhq_huff.so,pair3=build/v/lib_pair3.so,pair4=build/v/lib_pair4.so,pair2=build/v/lib_pair2.so \
  --check pair3,pair4,pair2 > "$OUT/ab_pair.txt" 2>&1 || { cat "$OUT/ab_pair.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_pair.txt"
