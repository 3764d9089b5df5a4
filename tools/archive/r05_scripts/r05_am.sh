#!/bin/bash
# Round 5 call am: the packed encode's mean bound (40 / 48 / 64 B) on config 4 and text of 44-54 B means.
set -o pipefail
OUT=${1:-gpurun_out/r05am}
mkdir -p "$OUT"
for v in pk48 pk64; do
  MHQ_LIB_PATH=build/v/lib_$v.so timeout -k 10 600 python3 -u -m pytest tests/test_encode_packed.py -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > "$OUT/tests_$v.txt" 2>&1 || { tail -30 "$OUT/tests_$v.txt"; exit 1; }
  echo "$v $(tail -1 "$OUT/tests_$v.txt")"
done
timeout -k 10 900 python3 tools/abmulti.py --kernel packed --reps 3 --configs config4,uniform:8:80,uniform:8:100 \
  --libs base=minhq_amd/libmhq_huff.so,pk48=build/v/lib_pk48.so,pk64=build/v/lib_pk64.so > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
