#!/bin/bash
# Round 5 call as: split (lengths only) code / length LDS tables in the staged encode (MHQ_ENC_SPLIT) A/B, encode tests.
set -o pipefail
OUT=${1:-gpurun_out/r05as}
mkdir -p "$OUT"
L=base=minhq_amd/libmhq_huff.so,split2=build/v/lib_split2.so
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --reps 3 --configs config2,northstar,config3 --libs $L > "$OUT/ab_packed.txt" 2>&1 || { cat "$OUT/ab_packed.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_packed.txt"
timeout -k 10 600 python3 tools/abmulti.py --kernel encode --reps 3 --configs config4,config2 --libs $L > "$OUT/ab_encode.txt" 2>&1 || { cat "$OUT/ab_encode.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_encode.txt"
MHQ_LIB_PATH=build/v/lib_split2.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_encode_packed.py tests/test_encode_groups.py tests/test_gpu_parity.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -3 "$OUT/tests.txt"
