#!/bin/bash
# Round 5 call v: paired steps by default -- GPU suite, read path and decode A/B against round-5 HEAD's build.
set -o pipefail
OUT=${1:-gpurun_out/r05v}
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/gpu_tests.txt" 2>&1 || { tail -30 "$OUT/gpu_tests.txt"; exit 1; }
tail -1 "$OUT/gpu_tests.txt"
timeout -k 10 600 python3 tools/ab_read.py --libs base=build/v/lib_steps3.so,pair=minhq_amd/libmhq_huff.so > "$OUT/ab_read.txt" 2>&1 || { cat "$OUT/ab_read.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_read.txt"
