#!/bin/bash
# r05: the AMDGPU scheduler's own register-pressure trackers (-mllvm -amdgpu-use-amdgpu-trackers=1;
# ab/trackers): tail<7, last> spills 91 -> 47 VGPRs, tail<7> 38 -> 32, head<6> 34 -> 32.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for cfg in metric c2 c4 c3; do
    run --label now --config $cfg
    DXRPT_KERNEL_LIB_DIR=ab/trackers run --label trackers --config $cfg
  done
  for rk in 2 5; do
    run --label now --share 8 --rank $rk --cur-copy
    DXRPT_KERNEL_LIB_DIR=ab/trackers run --label trackers --share 8 --rank $rk --cur-copy
  done
  run --label now --share 4 --rank 2 --cur-copy
  DXRPT_KERNEL_LIB_DIR=ab/trackers run --label trackers --share 4 --rank 2 --cur-copy
done
