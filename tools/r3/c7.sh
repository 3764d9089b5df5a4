#!/bin/bash
# headline launch path: HIP-graph replay vs direct ABI calls, 20 and 200 steps
set -o pipefail
mkdir -p gpurun_out/r3
for launch in graph direct; do
  for steps in 20 200; do
    timeout -k 10 300 python3 bench.py --steps $steps --warmup 5 --no-extras --no-cpu --launch $launch > gpurun_out/r3/b_${launch}_${steps}.json 2> gpurun_out/r3/b_${launch}_${steps}.err || { echo "FAIL $launch $steps"; tail -20 gpurun_out/r3/b_${launch}_${steps}.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r3/b_${launch}_${steps}.json')); print('$launch', $steps, d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'], d['encode_ms_per_launch'])"
  done
done
