#!/bin/bash
# GPU suite, smoke and the 20-step bench (the driver's shape): bash tools/r06/suite.sh OUT
set -o pipefail
OUT=${1:?}; mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/gpu_tests.txt" 2>&1 || { tail -40 "$OUT/gpu_tests.txt"; exit 1; }
tail -2 "$OUT/gpu_tests.txt"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 || { tail "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
timeout -k 10 900 python3 -u bench.py --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.log" || { tail -30 "$OUT/bench.log"; exit 1; }
python3 -c "
import json,sys; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms/step', d['ms_per_step'], 'long_run', (d.get('long_run') or {}).get('ms_per_step'))
print('decode_only_northstar', d.get('decode_only_northstar',{}).get('ms_per_launch'), d.get('decode_only_northstar',{}).get('hbm_frac'))
print('roofline', d['roofline']['kernel'], d['roofline']['ms_per_launch'], d['roofline']['frac'])
"
