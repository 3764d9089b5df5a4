#!/bin/bash
# Round-3 checkpoint on one box: GPU tests, then per-config kernel times of
# decode / encode / layout, then the bench (+ rocprof stats and PMC traffic).
set -o pipefail
OUT=${1:-gpurun_out/r3base}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -4 $OUT/gpu_tests.txt; [ $rc = 0 ] || exit $rc
for k in decode encode layout; do
  for cfg in northstar config2 config3 config2print config4 config5; do
    timeout -k 10 120 python3 tools/kernel_driver.py --kernel $k --config $cfg --iters 30 --no-check >> $OUT/configs.jsonl 2>$OUT/kd.err || { echo "kd $k $cfg failed"; tail $OUT/kd.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('$OUT/configs.jsonl'):
    d=json.loads(l); print(d.get('kernel'), d.get('config'), d.get('us_per_launch'), d.get('hbm_frac'))"
[ -n "$NOBENCH" ] && exit 0
bash tools/round_profile.sh $OUT/round
