#!/bin/bash
# Round 5 call ay: packed encode at four workgroups per CU: staging loads issued together (stg), 16-B sizing (sz16), both, look-back windows 2 / 8, A/B; tests of each changed form.
set -o pipefail
OUT=${1:-gpurun_out/r05ay}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --reps 3 --configs config2,northstar,config3 \
  --libs base=minhq_amd/libmhq_huff.so,stg=build/v/lib_stg.so,sz16=build/v/lib_sz16.so,both=build/v/lib_both.so,w2=build/v/lib_w2.so,w8=build/v/lib_w8.so > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
MHQ_LIB_PATH=build/v/lib_both.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_encode_packed.py > "$OUT/tests_both.txt" 2>&1 || { tail -30 "$OUT/tests_both.txt"; exit 1; }
tail -1 "$OUT/tests_both.txt"
