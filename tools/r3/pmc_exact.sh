#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the decode with exact-length output regions vs the capacity layout (north star)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcx
for mode in cap exact; do
  x=""; [ $mode = exact ] && x="--exact"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d gpurun_out/pmcx/${mode}_$ctr -o run -- python3 tools/kernel_driver.py --kernel decode --config northstar --iters 10 $x > gpurun_out/pmcx/${mode}_$ctr.log 2>&1 || { echo "pass $mode $ctr failed"; tail -5 gpurun_out/pmcx/${mode}_$ctr.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob
for mode in ("cap", "exact"):
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(f"gpurun_out/pmcx/{mode}_{ctr}/**/*counter_collection.csv", recursive=True)
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f[0])) if "decode_kernel" in r.get("Kernel_Name", "") and r.get("Counter_Name") == ctr]
        v = sorted(vals)[len(vals) // 2] if vals else float("nan")
        print(mode, ctr, "median KB per launch", round(v, 1), "launches", len(vals))
PY
