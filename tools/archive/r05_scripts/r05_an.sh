#!/bin/bash
# Round 5 call an: the decode without its counting sort (MHQ_DEC_NOSORT), A/B.
set -o pipefail
OUT=${1:-gpurun_out/r05an}
mkdir -p "$OUT"
timeout -k 10 900 python3 tools/abmulti.py --kernel decode --reps 3 --configs northstar,config2,config3,config4 \
  --libs base=minhq_amd/libmhq_huff.so,nosort=build/v/lib_nosort.so --check nosort > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt" | grep -v SAME
grep -c SAME "$OUT/ab.txt"
