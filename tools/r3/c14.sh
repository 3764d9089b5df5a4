#!/bin/bash
# decode phase priority A/B; read_strings / ints / varints rows (tools/bench_rows.py)
set -o pipefail
mkdir -p gpurun_out/r3
VDIR=tools/r3/v bash tools/r3/ab.sh "northstar config2 config3" decode prio0 prio1 || exit 1
timeout -k 10 300 python3 tools/bench_rows.py > gpurun_out/r3/rows.json 2> gpurun_out/r3/rows.err || { tail gpurun_out/r3/rows.err; exit 1; }
cat gpurun_out/r3/rows.json
