#!/bin/bash
# Round 5 call h: the packed encode with the one-wave look-back after the
# encode: its tests, then its time beside the split form and timing builds.
set -o pipefail
OUT=${1:-gpurun_out/r05h}
mkdir -p "$OUT"
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_encode_packed.py > "$OUT/packed_tests.txt" 2>&1 || { echo "packed tests failed"; tail -30 "$OUT/packed_tests.txt"; exit 1; }
tail -2 "$OUT/packed_tests.txt"
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --configs northstar,config2,config3 \
  --libs base=minhq_amd/libmhq_huff.so,nolb=build/v/lib_pk_nolb.so,noenc=build/v/lib_pk_noenc.so \
  > "$OUT/ab_packed_builds.txt" 2>&1 && \
timeout -k 10 600 python3 tools/abmulti.py --kernel layenc --configs northstar,config2,config3 \
  --libs base=minhq_amd/libmhq_huff.so > "$OUT/ab_layenc.txt" 2>&1 || { echo "ab failed"; tail -20 "$OUT/ab_packed_builds.txt"; exit 1; }
cat "$OUT/ab_packed_builds.txt" "$OUT/ab_layenc.txt"
