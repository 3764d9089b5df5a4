#!/bin/bash
# Round 5 call af: the long-literal form's shape (waves per workgroup, window size, workgroups per CU), config 5 sized.
set -o pipefail
OUT=${1:-gpurun_out/r05af}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_decode_long.py -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
for v in lw10x2 lw16w64; do
  MHQ_LIB_PATH=build/v/lib_$v.so timeout -k 10 600 python3 -u -m pytest tests/test_decode_long.py -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > "$OUT/tests_$v.txt" 2>&1 || { tail -30 "$OUT/tests_$v.txt"; exit 1; }
  echo "$v $(tail -1 "$OUT/tests_$v.txt")"
done
timeout -k 10 600 python3 tools/abmulti.py --kernel decode --configs config5 --reps 3 --sized \
  --libs base=minhq_amd/libmhq_huff.so,lw10x2=build/v/lib_lw10x2.so,lw16w64=build/v/lib_lw16w64.so,lw8x3=build/v/lib_lw8x3.so \
  --check lw10x2,lw16w64,lw8x3 > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v "amdgpu.ids" "$OUT/ab.txt"
