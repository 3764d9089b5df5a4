#!/bin/bash
# Round 3 A/B: decode parity tests on the default library, then decode timings
# of the default vs prebuilt variants (build/var/lib_<name>.so) on several configs.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_stream_path.py tests/test_strings.py} -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${CONFIGS:-northstar config2}; do
  for name in default "$@"; do
    lib=build/var/lib_$name.so; [ "$name" = default ] && lib=minhq_amd/libmhq_huff.so
    printf "%-10s " $name
    MHQ_LIB_PATH=$lib timeout -k 10 120 python3 tools/kernel_driver.py --kernel ${KERNEL:-decode} --config $cfg --iters 30 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
