#!/bin/bash
# r03: SBVH build variants (ab/bins64: 64 SAH bins; ab/alpha6 / ab/alpha4: spatial-split search threshold
# 1e-6 / 1e-4 of the root area) against the in-tree build (32 bins, 1e-5).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for cfg in "--config metric" "--config c4" "--config c5 --share 8 --rank 3" "--config c2" "--config metric --share 8 --rank 2"; do
  for b in dxrpathtracer_amd/lib ab/bins64 ab/alpha6 ab/alpha4; do
    DXRPT_KERNEL_LIB_DIR=$b timeout -k 10 240 python -u scripts/time_frames.py --rounds 3 --frames 24 $cfg --label $b 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
