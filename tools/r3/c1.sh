#!/bin/bash
# round-3 first call: loop microbenchmarks (1 vs 2 chains, waves/CU), then the baseline checkpoint
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 200 ./tools/ubench/ubench_loop 1000 > gpurun_out/r3/ubench_loop.txt 2>&1 || { cat gpurun_out/r3/ubench_loop.txt; exit 1; }
timeout -k 10 100 ./tools/ubench/ubench_lean 1000 > gpurun_out/r3/ubench_lean.txt 2>&1 || { cat gpurun_out/r3/ubench_lean.txt; exit 1; }
cat gpurun_out/r3/ubench_loop.txt gpurun_out/r3/ubench_lean.txt
bash tools/r3/base.sh gpurun_out/r3base
