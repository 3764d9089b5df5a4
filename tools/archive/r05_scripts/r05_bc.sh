#!/bin/bash
# Round 5 call bc: the packed encode's two shapes picked by the mean (four workgroups up to a 37.5-B mean, three above) against three always; packed tests.
set -o pipefail
OUT=${1:-gpurun_out/r05bc}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --reps 3 --configs config2,northstar,config3,uniform:24:56,uniform:30:46,uniform:36:44,zipf:4:96 \
  --libs pick=minhq_amd/libmhq_huff.so,pk3=build/v/lib_pk3.so > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_encode_packed.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
