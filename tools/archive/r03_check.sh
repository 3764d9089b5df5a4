set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for cfg in northstar config2; do
  timeout -k 10 120 python3 tools/kernel_driver.py --kernel decode --config $cfg --iters 30 2>&1 | grep -v amdgpu.ids || exit 1
done
