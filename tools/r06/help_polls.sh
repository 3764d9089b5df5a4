#!/bin/bash
# The driver's short bench (20 steps, 5 warm-up) at look-back help thresholds
# (MHQ_PK_HELP_POLLS, read once per process), interleaved: bash tools/r06/help_polls.sh OUT
set -o pipefail
OUT=${1:?}; mkdir -p "$OUT"
for r in 1 2 3; do
  for p in 400 100 25; do
    MHQ_PK_HELP_POLLS=$p timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu --no-configs \
      > "$OUT/b_${p}_$r.json" 2> "$OUT/b_${p}_$r.err" || { tail "$OUT/b_${p}_$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" "$OUT/b_${p}_$r.json" "polls=$p rep=$r"
  done
done
