#!/bin/bash
# r03: confirm ab/hp2 (depth-1 sun shadow packets two triangles at a time) against the in-tree build, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in 1 2 3; do
  for cfg in "--config metric" "--config c4" "--config metric --share 8 --rank 2"; do
    for b in dxrpathtracer_amd/lib ab/hp2; do
      DXRPT_KERNEL_LIB_DIR=$b timeout -k 10 240 python -u scripts/time_frames.py --rounds 3 --frames 32 $cfg --label $b 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done
