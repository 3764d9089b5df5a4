#!/bin/bash
# Round 5 call be: where the layout call's scan pass goes (timing builds: no prefix of the sums before a chunk, no stores; the three-pass form), A/B.
set -o pipefail
OUT=${1:-gpurun_out/r05be}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel layout --reps 3 --configs config2,northstar \
  --libs base=minhq_amd/libmhq_huff.so,xs1=build/v/lib_xs1.so,xs2=build/v/lib_xs2.so,nodirect=build/v/lib_nodirect.so > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
