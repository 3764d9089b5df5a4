#!/bin/bash
# Round 5 call bf: the one-launch layout (encode_len with a look-back, mhq_huff_encode_layout_sized_dev): layout parity tests first, then A/B against the two-launch call.
set -o pipefail
OUT=${1:-gpurun_out/r05bf}
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "layout or round_trip" > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
timeout -k 10 600 python3 tools/abmulti.py --kernel layout --reps 3 --configs config2,northstar,config3,config4 \
  --libs two=minhq_amd/libmhq_huff.so,one=minhq_amd/libmhq_huff.so --sized-layout one > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
