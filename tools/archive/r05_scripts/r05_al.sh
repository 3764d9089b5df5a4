#!/bin/bash
# Round 5 call al: the decode kernel (tiles, pieces, streamed tiles) against the long-literal form on long text means, sized.
set -o pipefail
OUT=${1:-gpurun_out/r05al}
mkdir -p "$OUT"
timeout -k 10 900 python3 tools/abmulti.py --kernel decode --reps 3 --sized \
  --configs uniform:32:160,uniform:64:192,uniform:128:256,uniform:256:512,config5 \
  --libs long=minhq_amd/libmhq_huff.so,tiles=build/v/lib_lmoff.so --check tiles > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt" | grep -v SAME
grep -c SAME "$OUT/ab.txt"
