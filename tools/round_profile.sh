#!/bin/bash
# One GPU call's worth of round evidence (run on the GPU box):
#   1. bench.py (default config, CPU baseline)           -> $OUT/bench.json
#   2. rocprofv3 --kernel-trace --stats of the same bench -> $OUT/stats/
#   3. FETCH_SIZE and WRITE_SIZE passes (separate runs)  -> $OUT/pmc_fetch, $OUT/pmc_write
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/round}
mkdir -p "$OUT"
BENCH="bench.py"
timeout -k 10 600 python3 $BENCH --cpu-seconds 15 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 $BENCH --no-cpu --no-extras \
  > "$OUT/stats.log" 2>&1 || { echo "stats pass failed"; tail "$OUT/stats.log"; exit 1; }
echo "stats ok"
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 $BENCH --no-cpu --no-extras \
  > "$OUT/pmc_fetch.log" 2>&1 || { echo "fetch pass failed"; tail "$OUT/pmc_fetch.log"; exit 1; }
echo "fetch ok"
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 $BENCH --no-cpu --no-extras \
  > "$OUT/pmc_write.log" 2>&1 || { echo "write pass failed"; tail "$OUT/pmc_write.log"; exit 1; }
echo "write ok"
