#!/bin/bash
# Round 5 call p: the packed encode's per-workgroup phase timeline (MHQ_DIAG_PKTL build).
set -o pipefail
OUT=${1:-gpurun_out/r05p}
mkdir -p "$OUT"
for cfg in northstar config2; do
  MHQ_LIB_PATH=build/v/lib_pktl.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel packed --config $cfg --iters 20 \
    > "$OUT/pktl_$cfg.txt" 2>&1 || { cat "$OUT/pktl_$cfg.txt"; exit 1; }
  timeout -k 10 120 python3 tools/kernel_driver.py --kernel packed --config $cfg --iters 50 >> "$OUT/pktl_$cfg.txt" 2>&1 || exit 1
  grep -v amdgpu.ids "$OUT/pktl_$cfg.txt"
done
