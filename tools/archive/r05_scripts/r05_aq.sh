#!/bin/bash
# Round 5 call aq: packed encode ranges sized to fill whole generations (MHQ_PK_FILL) A/B, timeline, packed tests.
set -o pipefail
OUT=${1:-gpurun_out/r05aq}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --reps 3 --configs config2,config4,northstar,config3 \
  --libs fill=minhq_amd/libmhq_huff.so,nofill=build/v/lib_nofill.so --check nofill > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt" | grep -v SAME
grep -c SAME "$OUT/ab.txt"
MHQ_LIB_PATH=build/v/lib_pktl.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel packed --config config2 --iters 20 > "$OUT/pktl.txt" 2>&1 || { cat "$OUT/pktl.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/pktl.txt"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_encode_packed.py tests/test_encode_groups.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -3 "$OUT/tests.txt"
