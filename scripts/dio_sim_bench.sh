#!/bin/bash
# The daemon-shaped loop end to end (files read from the page cache, pinned
# windows over PCIe, one update_batch per wakeup): fdfs_dio_sim over 2,048
# files of U[0.25, 2] MiB at 64 / 1,024 uploads in flight, each method.
set -o pipefail
mkdir -p gpurun_out
D=$(mktemp -d /tmp/dio_sim.XXXXXX)
python - "$D" <<'PY'
import sys, numpy as np
d = sys.argv[1]
rng = np.random.default_rng(7)
for i, n in enumerate(rng.integers(1 << 18, 2 << 20, 2048)):
    rng.integers(0, 256, int(n), dtype=np.uint8).tofile(f"{d}/f{i:05d}")
PY
for m in crc hash md5; do
  for j in 64 1024; do
    echo -n "method $m jobs $j: "
    timeout -k 10 120 ./fastdfs_amd/lib/fdfs_dio_sim -m $m -j $j $D/f* 2>&1 >/dev/null | tail -1 || exit 1
  done
done
rm -rf "$D"
