#!/bin/bash
# A/B: packet triangles staged in LDS (in-tree build) vs scalar loads (ab/nostage).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 200 python -u scripts/time_frames.py --rounds 3 --frames 24"
for r in 1 2; do
for b in dxrpathtracer_amd/lib ab/nostage; do
  for args in "--config metric" "--config c4" "--config c2" "--config c3" "--config metric --share 8 --rank 5" "--config metric --share 8 --rank 2" "--config metric --share 4 --rank 1" "--config metric --share 2 --rank 1"; do
    DXRPT_KERNEL_LIB_DIR=$b $T $args --label $b 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
done
