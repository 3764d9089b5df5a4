#!/bin/bash
# Round 5 call ag: the streamed path touching each literal's next window a round ahead (MHQ_DEC_LONG_TOUCH), config 5 / 4.
set -o pipefail
OUT=${1:-gpurun_out/r05ag}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel decode --configs config5,config4 --reps 3 --sized \
  --libs base=minhq_amd/libmhq_huff.so,touch=build/v/lib_touch.so --check touch > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v "amdgpu.ids" "$OUT/ab.txt"
