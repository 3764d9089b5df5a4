set -o pipefail
mkdir -p gpurun_out
for v in ${TLV:-tl count}; do
  echo "== $v"
  MHQ_LIB_PATH=build/var/lib_$v.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel decode --config ${CFG:-northstar} --iters 20 --no-check 2>&1 | grep -v amdgpu.ids || exit 1
done
