#!/bin/bash
# Round 5 call s: packed encode straight to global memory (MHQ_PK_DIRECT=1, five workgroups per CU)
# against the staged form -- tests, timing, timeline.
set -o pipefail
OUT=${1:-gpurun_out/r05s}
mkdir -p "$OUT"
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_encode_packed.py > "$OUT/packed_tests.txt" 2>&1 || { tail -30 "$OUT/packed_tests.txt"; exit 1; }
tail -2 "$OUT/packed_tests.txt"
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --configs northstar,config2,config3 \
  --libs direct=minhq_amd/libmhq_huff.so,staged=build/v/lib_pkstage.so > "$OUT/ab_packed.txt" 2>&1 || { cat "$OUT/ab_packed.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_packed.txt"
MHQ_LIB_PATH=build/v/lib_pktl.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel packed --config northstar --iters 20 \
  > "$OUT/pktl_northstar.txt" 2>&1 || { cat "$OUT/pktl_northstar.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/pktl_northstar.txt"
