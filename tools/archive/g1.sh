set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream_path.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt1.log 2>&1
rc=$?; tail -5 gpurun_out/pt1.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="${CONFIGS:-northstar config2}" bash tools/var_times.sh default $VARIANTS
