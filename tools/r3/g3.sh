#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 100 ./tools/ubench/ubench_lean 1000 > gpurun_out/r3/ubench_lean.txt 2>&1 || { cat gpurun_out/r3/ubench_lean.txt; exit 1; }
timeout -k 10 100 ./tools/ubench/ubench_loop 1000 > gpurun_out/r3/ubench_loop3.txt 2>&1 || { cat gpurun_out/r3/ubench_loop3.txt; exit 1; }
cat gpurun_out/r3/ubench_lean.txt gpurun_out/r3/ubench_loop3.txt
