#!/bin/bash
# Round 5 call b: r05_fault.sh, then the byte-store decode variant (MHQ_DEC_BW):
# the decode/read GPU tests on its bounds build, then an A/B of the decode
# kernel against the product library (outputs compared).
set -o pipefail
OUT=${1:-gpurun_out/r05b}
mkdir -p "$OUT"
bash tools/r05_fault.sh "$OUT" || exit 1
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 env MHQ_LIB_PATH=build/v/lib_bw_dbg.so MHQ_DBG_BOUNDS_CHECK=1 $T tests/test_gpu_parity.py \
  tests/test_gpu_stream_path.py tests/test_strings.py tests/test_headers.py > "$OUT/bw_dbg_tests.txt" 2>&1 \
  || { echo "bw bounds tests failed rc=$?"; tail -30 "$OUT/bw_dbg_tests.txt"; exit 1; }
tail -2 "$OUT/bw_dbg_tests.txt"
timeout -k 10 600 python3 tools/abmulti.py --kernel decode --configs northstar,config2,config3,config2print,config5 \
  --libs base=minhq_amd/libmhq_huff.so,bw=build/v/lib_bw.so,bw4=build/v/lib_bw4.so --check bw,bw4 --reps 3 \
  > "$OUT/ab_bw.txt" 2>&1 || { echo "ab failed"; tail -20 "$OUT/ab_bw.txt"; exit 1; }
cat "$OUT/ab_bw.txt"
timeout -k 10 600 python3 tools/abmulti.py --kernel layenc --configs northstar,config2,config3 \
  --libs base=minhq_amd/libmhq_huff.so > "$OUT/ab_layenc.txt" 2>&1 && \
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --configs northstar,config2,config3 \
  --libs base=minhq_amd/libmhq_huff.so > "$OUT/ab_packed.txt" 2>&1 || { echo "packed ab failed"; tail -20 "$OUT/ab_packed.txt"; exit 1; }
cat "$OUT/ab_layenc.txt" "$OUT/ab_packed.txt"
