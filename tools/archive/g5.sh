# GPU tests (all), then the row measurements
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_all.log 2>&1
rc=$?; tail -5 gpurun_out/pt_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/bench_rows.py 2>&1 | grep -v amdgpu.ids
