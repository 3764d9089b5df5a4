#!/bin/bash
# Final round check on one GPU: all -m gpu tests, smoke(), default bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final/pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/final/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.txt 2>&1 || { tail gpurun_out/final/smoke.txt; exit 1; }
tail -1 gpurun_out/final/smoke.txt
timeout -k 10 600 python3 bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail gpurun_out/final/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/final/bench.json')); print(d['value'], d['roofline']['frac'], d['decode_only_northstar']['hbm_frac'])"
