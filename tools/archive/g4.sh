# parity tests on a variant library, then timings: VAR=name bash tools/g4.sh
set -o pipefail
mkdir -p gpurun_out
MHQ_LIB_PATH=build/var/lib_$VAR.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream_path.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_$VAR.log 2>&1
rc=$?; tail -5 gpurun_out/pt_$VAR.log; [ $rc -eq 0 ] || exit $rc
CONFIGS="${CONFIGS:-northstar config2}" bash tools/var_times.sh default $VAR default $VAR
