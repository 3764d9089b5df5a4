#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
MHQ_LIB_PATH=tools/r3/dbgv/lib_dbg.so timeout -k 10 120 python -u tools/r3/encdbg.py > gpurun_out/encdbg2.log 2>&1
