#!/bin/bash
# Round 5 call ba: the thread-form encode at four workgroups per CU (MHQ_ENC_BLOCKS 4, 19.4-KB / 15-KB staging, 64 VGPRs) A/B, encode tests.
set -o pipefail
OUT=${1:-gpurun_out/r05ba}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel encode --reps 3 --configs config4,config2,northstar,uniform:40:120,uniform:64:128 \
  --libs t3=minhq_amd/libmhq_huff.so,t4=build/v/lib_t4.so > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
MHQ_LIB_PATH=build/v/lib_t4.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_encode_groups.py tests/test_gpu_parity.py tests/test_encode_packed.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
