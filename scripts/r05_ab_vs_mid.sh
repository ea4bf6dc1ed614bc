#!/bin/bash
# r05: the current build against the mid-round build (ab/r05mid = commit 799839b: chained shadows,
# branch-free texels; before the 115 % budget, three frames in flight, split threshold, head 6 and packed
# taps), same box, interleaved -- box-to-box spread is ~2 %, so cross-commit gains are measured here.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for cfg in metric c2 c4 c3; do
    run --label now --config $cfg --kernels
    DXRPT_KERNEL_LIB_DIR=ab/r05mid run --label r05mid --config $cfg --kernels
  done
  run --label now --config c5 --rounds 3 --frames 8
  DXRPT_KERNEL_LIB_DIR=ab/r05mid run --label r05mid --config c5 --rounds 3 --frames 8
  for rk in 2 5; do
    run --label now --share 8 --rank $rk --cur-copy
    DXRPT_KERNEL_LIB_DIR=ab/r05mid run --label r05mid --share 8 --rank $rk --cur-copy
  done
done
