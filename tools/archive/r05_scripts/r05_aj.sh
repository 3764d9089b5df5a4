#!/bin/bash
# Round 5 call aj: the thread form up to a 96-B mean -- encode tests, encode A/B against HEAD across shapes.
set -o pipefail
OUT=${1:-gpurun_out/r05aj}
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_encode_packed.py tests/test_strings.py -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
timeout -k 10 900 python3 tools/abmulti.py --kernel encode --reps 3 \
  --configs northstar,config2,config3,config4,uniform:8:80,uniform:32:160,uniform:64:192,config5 \
  --libs head=build/v/lib_headenc.so,new=minhq_amd/libmhq_huff.so > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
