#!/bin/bash
# Round 5 call g: where the packed encode's time goes (timing builds: no
# look-back wait, no encode, no sizing pass), beside the split form.
set -o pipefail
OUT=${1:-gpurun_out/r05g}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --configs northstar,config2 \
  --libs base=minhq_amd/libmhq_huff.so,nolb=build/v/lib_pk_nolb.so,noenc=build/v/lib_pk_noenc.so,nosize=build/v/lib_pk_nosize.so \
  > "$OUT/ab_packed_builds.txt" 2>&1 || { echo "ab failed"; tail -20 "$OUT/ab_packed_builds.txt"; exit 1; }
cat "$OUT/ab_packed_builds.txt"
timeout -k 10 600 python3 tools/abmulti.py --kernel encode --configs northstar,config2 \
  --libs base=minhq_amd/libmhq_huff.so > "$OUT/ab_encode.txt" 2>&1 && \
timeout -k 10 600 python3 tools/abmulti.py --kernel layout --configs northstar,config2 \
  --libs base=minhq_amd/libmhq_huff.so > "$OUT/ab_layout.txt" 2>&1 || { echo "ab2 failed"; exit 1; }
cat "$OUT/ab_encode.txt" "$OUT/ab_layout.txt"
