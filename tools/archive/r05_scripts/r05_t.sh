#!/bin/bash
# Round 5 call t: decode PMC counters (issue, LDS, waits) for the long-literal shapes (configs 5 and 4) and the north star.
set -o pipefail
OUT=${1:-gpurun_out/r05t}
mkdir -p "$OUT"
for cfg in config5 config4 northstar; do
  bash tools/prof_pmc_lds.sh "$OUT/$cfg" -- python3 tools/kernel_driver.py --kernel decode --config $cfg --iters 10 || exit 1
  python3 tools/pmc_summary.py "$OUT/$cfg" decode_kernel > "$OUT/${cfg}_summary.txt"
  cat "$OUT/${cfg}_summary.txt"
done
timeout -k 10 300 python3 tools/abmulti.py --kernel decode --configs config5,config4 --libs base=minhq_amd/libmhq_huff.so > "$OUT/ab_long.txt" 2>&1 || exit 1
grep -v amdgpu.ids "$OUT/ab_long.txt"
