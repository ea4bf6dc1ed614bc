#!/bin/bash
# r03: traversal pipelining (traverse8_pipe: bit 0 triangle pairs, bit 1 next-node prefetch) in the split
# schedule's per-lane closest hit (ab/ch*) and shadow rays (ab/ah*), against the in-tree build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for cfg in "--config metric" "--config c4" "--config c5 --share 8 --rank 3" "--config c3"; do
  for b in dxrpathtracer_amd/lib ab/ch1 ab/ch2 ab/ch3 ab/ah1 ab/ah2; do
    DXRPT_KERNEL_LIB_DIR=$b timeout -k 10 200 python -u scripts/time_frames.py --rounds 3 --frames 32 $cfg --label $b 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
