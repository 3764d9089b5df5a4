# parity of each variant library, then interleaved timings: VARS="a b" bash tools/g6.sh
set -o pipefail
mkdir -p gpurun_out
for v in $VARS; do
  MHQ_LIB_PATH=build/var/lib_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream_path.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 gpurun_out/pt_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
CONFIGS="${CONFIGS:-northstar config2}" bash tools/var_times.sh default $VARS default $VARS
