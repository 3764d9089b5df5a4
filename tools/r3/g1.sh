#!/bin/bash
# round 3, first GPU call: loop ubench + current decode baseline + timeline
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 120 ./tools/ubench/ubench_loop 1000 > gpurun_out/r3/ubench_loop.txt 2>&1 || { cat gpurun_out/r3/ubench_loop.txt; exit 1; }
cat gpurun_out/r3/ubench_loop.txt
timeout -k 10 180 python3 tools/kernel_driver.py --kernel decode --config northstar --iters 30 > gpurun_out/r3/base_ns.json 2>&1 || { cat gpurun_out/r3/base_ns.json; exit 1; }
cat gpurun_out/r3/base_ns.json
bash tools/diag_timeline.sh > gpurun_out/r3/tl.txt 2>&1 || { cat gpurun_out/r3/tl.txt; exit 1; }
cat gpurun_out/r3/tl.txt
