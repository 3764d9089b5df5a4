#!/bin/bash
# The read kernels without calls / flat LDS / scratch: the GPU suite, then
# read_strings old vs new (tools/ab_read.py): bash tools/r06/readfix.sh OUT
set -o pipefail
OUT=${1:?}; mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/gpu_tests.txt" 2>&1 || { tail -40 "$OUT/gpu_tests.txt"; exit 1; }
tail -2 "$OUT/gpu_tests.txt"
timeout -k 10 600 python3 -u tools/ab_read.py --libs head=build/r06v/lib_head.so,new=build/r06v/lib_new.so,head2=build/r06v/lib_head.so,new2=build/r06v/lib_new.so \
  --reps 3 > "$OUT/ab_read.txt" 2>&1 || { tail -20 "$OUT/ab_read.txt"; exit 1; }
grep -v "^$" "$OUT/ab_read.txt" | grep -v amdgpu.ids
