#!/bin/bash
# r03: alpha-tested triangle test priced 2x / 3x an opaque one in the BVH8 collapse (ab/ac2, ab/ac3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for cfg in "--config c4" "--config metric" "--config c5 --share 8 --rank 3" "--config c2" "--config metric --share 8 --rank 2" "--config metric --share 8 --rank 1"; do
  for b in dxrpathtracer_amd/lib ab/ac2 ab/ac3; do
    DXRPT_KERNEL_LIB_DIR=$b timeout -k 10 240 python -u scripts/time_frames.py --rounds 3 --frames 24 $cfg --label $b 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
