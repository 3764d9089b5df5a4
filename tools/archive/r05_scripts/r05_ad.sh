#!/bin/bash
# Round 5 call ad: packed encode with wave 0's look-back before its encode share -- tests, A/B against HEAD, timeline.
set -o pipefail
OUT=${1:-gpurun_out/r05ad}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_encode_packed.py -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --configs northstar,config2,config3 --reps 4 \
  --libs head=build/v/lib_head.so,new=minhq_amd/libmhq_huff.so > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v "amdgpu.ids" "$OUT/ab.txt"
MHQ_LIB_PATH=build/v/lib_pktl.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel packed --config northstar --iters 20 \
  > "$OUT/pktl.txt" 2>&1 || { cat "$OUT/pktl.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/pktl.txt"
