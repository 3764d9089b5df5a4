#!/bin/bash
# Round 5 call j: the whole GPU suite on 3-step read groups (current source),
# then the read path timed against the 2-step default.
set -o pipefail
OUT=${1:-gpurun_out/r05j}
mkdir -p "$OUT"
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 env MHQ_LIB_PATH=build/v/lib_steps3.so $T tests -m gpu > "$OUT/suite_steps3.txt" 2>&1 &&
timeout -k 10 600 python3 tools/ab_read.py --libs base=minhq_amd/libmhq_huff.so,steps3=build/v/lib_steps3.so \
  > "$OUT/ab_read.txt" 2>&1
rc=$?
tail -3 "$OUT/suite_steps3.txt"; cat "$OUT/ab_read.txt" | grep -v amdgpu.ids
exit $rc
