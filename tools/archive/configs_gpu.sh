#!/bin/bash
# Decode / encode / layout-call timings over the BASELINE configs (GPU box).
set -o pipefail
for k in decode encode layout; do
  for cfg in northstar config2 config2print config3 config4 config5; do
    timeout -k 10 200 python3 tools/kernel_driver.py --kernel $k --config $cfg --iters 10 2>/dev/null || { echo "$k $cfg failed"; exit 1; }
  done
done
