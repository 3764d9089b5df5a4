#!/bin/bash
# Round 5 call z: the decode's per-wave timeline (MHQ_DIAG_TIMELINE) on the north star and config 2, paired steps.
set -o pipefail
OUT=${1:-gpurun_out/r05z}
mkdir -p "$OUT"
for cfg in northstar config2; do
  MHQ_LIB_PATH=build/v/lib_tl.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel decode --config $cfg --iters 20 \
    > "$OUT/tl_$cfg.txt" 2>&1 || { cat "$OUT/tl_$cfg.txt"; exit 1; }
  grep -v amdgpu.ids "$OUT/tl_$cfg.txt"
done
