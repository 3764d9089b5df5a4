set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
PARITY_VARIANTS= KERNEL=encode CONFIGS="northstar config2 config4" bash tools/r03_abv.sh branchy || exit 1
PARITY_VARIANTS= KERNEL=layout CONFIGS="config2 config4" bash tools/r03_abv.sh nodirect || exit 1
