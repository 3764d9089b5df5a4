#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 200 ./tools/ubench/ubench_loop 1000 > gpurun_out/r3/ubench_loop2.txt 2>&1; rc=$?
cat gpurun_out/r3/ubench_loop2.txt; exit $rc
