set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/diag1
bash tools/variants.sh gpurun_out/diag1/v stamps=-DMHQ_DIAG_STAMPS nodec=-DMHQ_DIAG_NO_DECODE > gpurun_out/diag1/build.log 2>&1 || { echo build failed; tail gpurun_out/diag1/build.log; exit 1; }
for v in stamps nodec; do
  MHQ_LIB_PATH=gpurun_out/diag1/v/lib_$v.so timeout -k 10 120 python3 tools/kernel_driver.py --kernel decode --config northstar --iters 30 --no-check > gpurun_out/diag1/$v.json 2> gpurun_out/diag1/$v.err || { echo "$v failed"; tail gpurun_out/diag1/$v.err; exit 1; }
  echo "== $v"; cat gpurun_out/diag1/$v.json; grep diag gpurun_out/diag1/$v.err
done
timeout -k 10 120 python3 tools/kernel_driver.py --kernel decode --config northstar --iters 30 > gpurun_out/diag1/base.json 2>&1 && cat gpurun_out/diag1/base.json
bash tools/prof_pmc_lds.sh gpurun_out/diag1/pmc -- python3 tools/kernel_driver.py --kernel decode --config northstar --iters 10 && python3 tools/pmc_summary.py gpurun_out/diag1/pmc decode
