#!/bin/bash
# Round 5 last check of the final tree: GPU suite (with the 448-range edge tests), smoke, the driver's 20-step bench line.
set -o pipefail
OUT=${1:-gpurun_out/r05final8}
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/gpu_tests.txt" 2>&1 || { tail -30 "$OUT/gpu_tests.txt"; exit 1; }
tail -1 "$OUT/gpu_tests.txt"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 || { tail "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench20.json" 2> "$OUT/bench20.err" || { tail "$OUT/bench20.err"; exit 1; }
cut -c1-200 "$OUT/bench20.json"
