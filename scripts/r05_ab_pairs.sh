#!/bin/bash
# r05: material taps in pairs (eight texel loads issued together) in the head and low-occupancy k_path:
# ab/pair1 normal + albedo, ab/pair2 also metallic + roughness; head at 5 (default) and 4 waves/SIMD.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 120 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for cfg in metric c4; do
    run --label base --config $cfg --kernels
    for v in 1 2; do DXRPT_KERNEL_LIB_DIR=ab/pair$v run --label pair$v --config $cfg --kernels; done
    for v in 1 2; do DXRPT_KERNEL_LIB_DIR=ab/pair$v run --label pair$v-head4 --config $cfg --opt MEGAKERNEL_OCCUPANCY=4 --opt TAIL_OCCUPANCY=7; done
  done
  run --label base --share 8 --rank 2
  for v in 1 2; do DXRPT_KERNEL_LIB_DIR=ab/pair$v run --label pair$v --share 8 --rank 2; done
done
