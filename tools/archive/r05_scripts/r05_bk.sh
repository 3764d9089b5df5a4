#!/bin/bash
# Round 5 call bk: packed encode stores: enc_len right after the range's scan (el), out_off / cap_off as streaming stores (nt), both; A/B and packed tests of both.
set -o pipefail
OUT=${1:-gpurun_out/r05bk}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --reps 5 --configs config2,northstar,config3 \
  --libs base=minhq_amd/libmhq_huff.so,el=build/v/lib_el.so,nt=build/v/lib_nt.so,both=build/v/lib_both.so > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
MHQ_LIB_PATH=build/v/lib_both.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_encode_packed.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
