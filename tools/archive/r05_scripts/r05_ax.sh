#!/bin/bash
# Round 5 call ax: the packed encode at four workgroups per CU (MHQ_PK_BLOCKS 4: 20-KB / 15-KB staging, the sort in the output staging) A/B, timeline, tests.
set -o pipefail
OUT=${1:-gpurun_out/r05ax}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --reps 3 --configs config2,northstar,config3,uniform:8:72 \
  --libs pk3=minhq_amd/libmhq_huff.so,pk4=build/v/lib_pk4.so > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
MHQ_LIB_PATH=build/v/lib_pktl4.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel packed --config config2 --iters 20 > "$OUT/pktl.txt" 2>&1 || { cat "$OUT/pktl.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/pktl.txt"
MHQ_LIB_PATH=build/v/lib_pk4.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_encode_packed.py > "$OUT/tests4.txt" 2>&1 || { tail -30 "$OUT/tests4.txt"; exit 1; }
tail -1 "$OUT/tests4.txt"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_encode_packed.py > "$OUT/tests3.txt" 2>&1 || { tail -30 "$OUT/tests3.txt"; exit 1; }
tail -1 "$OUT/tests3.txt"
