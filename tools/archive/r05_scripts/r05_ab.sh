#!/bin/bash
# Round 5 call ab: the first tile's sort overlapping its input loads (stage after the sort) against HEAD; decode tests.
set -o pipefail
OUT=${1:-gpurun_out/r05ab}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_strings.py -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
timeout -k 10 600 python3 tools/abmulti.py --kernel decode --configs northstar,config2,config3,config2print --reps 4 \
  --libs head=build/v/lib_head.so,new=minhq_amd/libmhq_huff.so --check new > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v "amdgpu.ids" "$OUT/ab.txt"
