#!/bin/bash
# Round 6 GPU runs: bash tools/r06/run.sh OUT STEP...   (steps: ab, ab4, tests, bench, prof)
set -o pipefail
OUT=${1:?out dir}; shift
mkdir -p "$OUT"
for step in "$@"; do
  case "$step" in
    ab) timeout -k 10 300 python3 -u tools/decode_ab.py --configs northstar,config2,config3,config2print --forms tile,stream \
          > "$OUT/ab.txt" 2>&1 || { tail -30 "$OUT/ab.txt"; exit 1; } ; cat "$OUT/ab.txt" ;;
    ab4) timeout -k 10 300 python3 -u tools/decode_ab.py --configs config4,config5 --n 1048576 --forms tile,stream \
          > "$OUT/ab4.txt" 2>&1 || { tail -30 "$OUT/ab4.txt"; exit 1; } ; cat "$OUT/ab4.txt" ;;
    tests) timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
          > "$OUT/gpu_tests.txt" 2>&1 || { tail -40 "$OUT/gpu_tests.txt"; exit 1; } ; tail -3 "$OUT/gpu_tests.txt" ;;
    bench) timeout -k 10 600 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.log" || { tail -30 "$OUT/bench.log"; exit 1; } ; cat "$OUT/bench.json" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
