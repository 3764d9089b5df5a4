#!/bin/bash
# Round 5 call bd: unstaged packed ranges reading aligned dwords (MHQ_PK_GW / MHQ_ENC_GW) A/B, forced four-workgroup shape for all-unstaged ranges; encode tests.
set -o pipefail
OUT=${1:-gpurun_out/r05bd}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --reps 3 --configs uniform:24:56,zipf:4:96,config2 \
  --libs gw=minhq_amd/libmhq_huff.so,gw0=build/v/lib_gw0.so,f4=build/v/lib_f4.so,f4gw0=build/v/lib_f4gw0.so > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
MHQ_LIB_PATH=build/v/lib_f4.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_encode_packed.py > "$OUT/tests_f4.txt" 2>&1 || { tail -30 "$OUT/tests_f4.txt"; exit 1; }
tail -1 "$OUT/tests_f4.txt"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_encode_packed.py tests/test_encode_groups.py tests/test_gpu_parity.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
