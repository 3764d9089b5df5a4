#!/bin/bash
# Packed encode with the compact code tables: its tests, then cpk0 vs cpk1 timing: bash tools/r06/cpk.sh OUT
set -o pipefail
OUT=${1:?}; mkdir -p "$OUT"
MHQ_LIB_PATH=build/r06v/lib_cpk2.so timeout -k 10 400 python3 -u -m pytest tests/test_encode_packed.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
timeout -k 10 400 python3 -u tools/abmulti.py --kernel packed --configs config2,northstar \
  --libs cpk0=build/r06v/lib_cpk0.so,cpk2=build/r06v/lib_cpk2.so,cpk0b=build/r06v/lib_cpk0.so,cpk2b=build/r06v/lib_cpk2.so \
  --reps 5 > "$OUT/ab.txt" 2>&1 || { tail -20 "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
