#!/bin/bash
# Per-wave timeline of the decode kernel (MHQ_DIAG_TIMELINE builds).
# Build here (CPU):  bash tools/abvar.sh build/v tl=-DMHQ_DIAG_TIMELINE [tl_x="-DMHQ_DIAG_TIMELINE -D..."]
# Run on the GPU box: bash tools/diag_timeline.sh build/v/lib_tl.so [more libs] [CONFIG=northstar]
set -o pipefail
cfg=${CONFIG:-northstar}
for lib in "$@"; do
  echo "== $lib ($cfg)"
  MHQ_LIB_PATH=$lib timeout -k 10 120 python3 tools/kernel_driver.py --kernel decode --config "$cfg" --iters 20 || exit 1
done
