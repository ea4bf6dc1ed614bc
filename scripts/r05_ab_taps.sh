#!/bin/bash
# r05 A/B, same box, interleaved: branch-free texel addressing (a bilinear tap's four loads issue together,
# in-tree) against ab/prev (the four loads serialised behind the per-lane format branch).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 120 python -u scripts/time_frames.py --rounds 5 "$@" || exit $?; }
for r in 1 2; do
  for cfg in metric c4 c3 c2; do for b in ab/prev dxrpathtracer_amd/lib; do DXRPT_KERNEL_LIB_DIR=$b run --label $b --config $cfg --kernels; done; done
  for rk in 2 5; do for b in ab/prev dxrpathtracer_amd/lib; do DXRPT_KERNEL_LIB_DIR=$b run --label $b --share 8 --rank $rk; done; done
  for b in ab/prev dxrpathtracer_amd/lib; do DXRPT_KERNEL_LIB_DIR=$b run --label $b --share 4 --rank 1; done
  for b in ab/prev dxrpathtracer_amd/lib; do DXRPT_KERNEL_LIB_DIR=$b run --label $b --config c5 --share 8 --rank 3; done
done
