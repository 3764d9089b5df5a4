#!/bin/bash
# Round 5 call c: ONE guarded replay of the shuffled read block on the BW
# bounds build (the build that faulted in r05b), then the packed-encode tests
# and its A/B on the product library.
set -o pipefail
OUT=${1:-gpurun_out/r05c}
mkdir -p "$OUT"
timeout -k 10 300 env MHQ_LIB_PATH=build/v/lib_bw_dbg.so AMD_LOG_LEVEL=1 python3 -u tools/dbg/read_fault_repro.py shuffled \
  > "$OUT/repro_bw_dbg_shuffled.txt" 2>&1
rc=$?
echo "repro rc=$rc"; tail -12 "$OUT/repro_bw_dbg_shuffled.txt"
grep -q "illegal memory access" "$OUT/repro_bw_dbg_shuffled.txt" && exit 1
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 env MHQ_LIB_PATH=build/v/lib_bw_dbg_inl.so python3 -u tools/dbg/read_fault_repro.py shuffled \
  > "$OUT/repro_bw_dbg_inl_shuffled.txt" 2>&1
rc=$?
echo "repro (helpers inlined) rc=$rc"; tail -6 "$OUT/repro_bw_dbg_inl_shuffled.txt"
grep -q "illegal memory access" "$OUT/repro_bw_dbg_inl_shuffled.txt" && exit 1
[ $rc -eq 0 ] || exit 1
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_encode_packed.py > "$OUT/packed_tests.txt" 2>&1 || { echo "packed tests failed"; tail -30 "$OUT/packed_tests.txt"; exit 1; }
tail -2 "$OUT/packed_tests.txt"
timeout -k 10 600 python3 tools/abmulti.py --kernel layenc --configs northstar,config2,config3 \
  --libs base=minhq_amd/libmhq_huff.so > "$OUT/ab_layenc.txt" 2>&1 && \
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --configs northstar,config2,config3 \
  --libs base=minhq_amd/libmhq_huff.so > "$OUT/ab_packed.txt" 2>&1 || { echo "packed ab failed"; tail -20 "$OUT/ab_packed.txt"; exit 1; }
cat "$OUT/ab_layenc.txt" "$OUT/ab_packed.txt"
