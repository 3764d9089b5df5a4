#!/bin/bash
# Round 5 call d: the byte-store decode (MHQ_DEC_BW) against the product
# decode, outputs compared, on the 2^20 shapes and config 5.
set -o pipefail
OUT=${1:-gpurun_out/r05d}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel decode --configs northstar,config2,config3,config2print,config5 \
  --libs base=minhq_amd/libmhq_huff.so,bw=build/v/lib_bw.so,bw4=build/v/lib_bw4.so --check bw,bw4 --reps 3 \
  > "$OUT/ab_bw.txt" 2>&1 || { echo "ab failed"; tail -20 "$OUT/ab_bw.txt"; exit 1; }
cat "$OUT/ab_bw.txt"
timeout -k 10 600 python3 tools/abmulti.py --kernel decode --configs northstar,config2 --exact \
  --libs base=minhq_amd/libmhq_huff.so,bw=build/v/lib_bw.so --check bw --reps 3 \
  > "$OUT/ab_bw_exact.txt" 2>&1 || { echo "ab exact failed"; tail -20 "$OUT/ab_bw_exact.txt"; exit 1; }
cat "$OUT/ab_bw_exact.txt"
