#!/bin/bash
# Round 5 evidence: the GPU suite, smoke(), then tools/round_profile.sh (bench, rocprof stats, FETCH/WRITE passes).
set -o pipefail
OUT=${1:-gpurun_out/r05final}
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/gpu_tests.txt" 2>&1 || { tail -30 "$OUT/gpu_tests.txt"; exit 1; }
tail -2 "$OUT/gpu_tests.txt"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 || { tail "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
bash tools/round_profile.sh "$OUT/round"
