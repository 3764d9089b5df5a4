#!/bin/bash
# Round 5 call au: the packed encode's look-back on a ninth wave with 448-literal ranges (MHQ_PK_LBWAVE, MHQ_PK_R) A/B, timeline, tests.
set -o pipefail
OUT=${1:-gpurun_out/r05au}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --reps 3 --configs config2,northstar,config3 \
  --libs lb0=build/v/lib_lb0.so,r448lb=build/v/lib_r448lb.so,r448=build/v/lib_r448.so > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
MHQ_LIB_PATH=build/v/lib_pktl.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel packed --config config2 --iters 20 > "$OUT/pktl.txt" 2>&1 || { cat "$OUT/pktl.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/pktl.txt"
MHQ_LIB_PATH=build/v/lib_r448lb.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_encode_packed.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -3 "$OUT/tests.txt"
