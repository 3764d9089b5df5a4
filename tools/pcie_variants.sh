#!/bin/bash
# PCIe-inclusive (host-memory ABI) rates of prebuilt variant libraries
# (build/var/lib_<name>.so; "default" = the in-tree build), config 2 batch.
set -o pipefail
for name in "$@"; do
  lib=build/var/lib_$name.so
  [ "$name" = default ] && lib=minhq_amd/libmhq_huff.so
  echo "== $name"
  MHQ_LIB_PATH=$lib timeout -k 10 150 python3 -c "
import bench, json
from minhq_amd import hc, workloads
b = workloads.make_batch(1 << 20, 'uniform', 'hdr', workloads.SEED_NORTH_STAR, 8, 64, 'config2')
with hc.Codec(devices=[0]) as c:
    print(json.dumps(bench.pcie_inclusive(c, b)))
" 2>&1 | grep -v amdgpu.ids || exit 1
done
