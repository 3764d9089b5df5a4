#!/bin/bash
# Round 6 evidence on the final code: GPU suite, smoke, north-star decode
# counters, then tools/round_profile.sh (bench, rocprof stats, FETCH/WRITE
# passes).  bash tools/r06/final.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r06final}
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/gpu_tests.txt" 2>&1 || { tail -30 "$OUT/gpu_tests.txt"; exit 1; }
tail -1 "$OUT/gpu_tests.txt"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 || { tail "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
bash tools/prof_pmc_lds.sh "$OUT/pmc_ns" -- python3 tools/kernel_driver.py --kernel decode --config northstar --iters 10 || exit 1
python3 tools/pmc_summary.py "$OUT/pmc_ns" decode_kernel > "$OUT/pmc_ns_summary.txt"
bash tools/round_profile.sh "$OUT/round"
