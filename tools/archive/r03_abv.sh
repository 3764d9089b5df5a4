#!/bin/bash
# Round 3 A/B with parity on the variants: decode parity tests on each variant
# library (MHQ_LIB_PATH), then decode timings of default vs variants, interleaved.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for name in ${PARITY_VARIANTS-"$@"}; do
  lib=build/var/lib_$name.so; [ "$name" = default ] && lib=minhq_amd/libmhq_huff.so
  MHQ_LIB_PATH=$lib timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_stream_path.py tests/test_strings.py} -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$name.log 2>&1
  rc=$?; echo "parity $name: $(tail -1 gpurun_out/pytest_$name.log)"; [ $rc -eq 0 ] || exit $rc
done
for cfg in ${CONFIGS:-northstar config2}; do
  for rep in 1 2; do
    for name in default "$@"; do
      lib=build/var/lib_$name.so; [ "$name" = default ] && lib=minhq_amd/libmhq_huff.so
      printf "%-10s " $name
      MHQ_LIB_PATH=$lib timeout -k 10 120 python3 -W ignore tools/kernel_driver.py --kernel ${KERNEL:-decode} --config $cfg --iters 30 2>&1 | grep -v amdgpu.ids | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['config'], d['us_per_launch'], d['hbm_frac'])" || exit 1
    done
  done
done
