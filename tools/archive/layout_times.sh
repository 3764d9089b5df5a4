#!/bin/bash
# Sizing + layout kernels on config 2: encode_len, the two-pass offsets scan,
# and the fused layout call (encode_len with block sums + one scan pass).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in encode_len offsets layout; do
  timeout -k 10 120 python3 tools/kernel_driver.py --kernel $k --config config2 --iters 50 2>/dev/null || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lay -o run -- \
  python3 tools/kernel_driver.py --kernel layout --config config2 --iters 50 > gpurun_out/lay.log 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/lay/run_kernel_stats.csv')):
    print(r['Name'][:50], r['Calls'], r['AverageNs'])
"
