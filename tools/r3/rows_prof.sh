#!/bin/bash
# Per-kernel times of the read_strings row (rocprofv3 kernel trace over tools/bench_rows.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rowsprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rowsprof -o rows -- python3 tools/bench_rows.py --blocks 200 > gpurun_out/rowsprof.log 2>&1 || { tail -20 gpurun_out/rowsprof.log; exit 1; }
tail -2 gpurun_out/rowsprof.log
f=$(find gpurun_out/rowsprof -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 "$f" | head -30
