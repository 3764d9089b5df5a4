#!/bin/bash
# Round 5 call y: packed encode ranges of 256 / 384 literals (more workgroups per CU) against 512.
set -o pipefail
OUT=${1:-gpurun_out/r05y}
mkdir -p "$OUT"
for v in pk256 pk384; do
  MHQ_LIB_PATH=build/v/lib_$v.so timeout -k 10 600 python3 -u -m pytest tests/test_encode_packed.py -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > "$OUT/tests_$v.txt" 2>&1 || { tail -20 "$OUT/tests_$v.txt"; exit 1; }
  echo "$v: $(tail -1 "$OUT/tests_$v.txt")"
done
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --configs northstar,config2,config3 --reps 4 \
  --libs base=minhq_amd/libmhq_huff.so,pk256=build/v/lib_pk256.so,pk384=build/v/lib_pk384.so > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v "amdgpu.ids" "$OUT/ab.txt"
