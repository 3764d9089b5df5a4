#!/bin/bash
# Round 5 call ae: the long-literal decode form (decode_long_kernel) -- tests, then config 5/4 timing (sized) against HEAD.
set -o pipefail
OUT=${1:-gpurun_out/r05ae}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_decode_long.py tests/test_gpu_parity.py -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
timeout -k 10 600 python3 tools/abmulti.py --kernel decode --configs config5,config4 --reps 3 --sized \
  --libs head=build/v/lib_headlong.so,new=minhq_amd/libmhq_huff.so > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v "amdgpu.ids" "$OUT/ab.txt"
