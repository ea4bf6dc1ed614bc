#!/bin/bash
# r04 A/B: the depth-split tails' shadow rays in their own kernel (k_path_tail_shadow, ab/tsh at 8 waves/SIMD,
# ab/tsh7 at 7), and closest hit + shading + shadows as three kernels (ab/t3; shading budget by option),
# against the in-tree build.  Parity of the variants first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in ab/tsh ab/t3; do
  DXRPT_KERNEL_LIB_DIR=$b timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
      -k "split or sponza_1080p_L8 or suntemple_alpha or white_furnace or settings_toggles or spot_lights" > gpurun_out/parity_${b#ab/}.log 2>&1
  echo "$b parity rc=$?"; tail -2 gpurun_out/parity_${b#ab/}.log
done
T="timeout -k 10 120 python -u scripts/time_frames.py --rounds 3 --kernels"
for cfg in "--config metric" "--config c3 --frames 16" "--config c4"; do
  for r in 1 2; do
    DXRPT_KERNEL_LIB_DIR=dxrpathtracer_amd/lib $T $cfg --label lib || exit 1
    DXRPT_KERNEL_LIB_DIR=ab/tsh $T $cfg --label tsh || exit 1
    DXRPT_KERNEL_LIB_DIR=ab/tsh7 $T $cfg --label tsh7 || exit 1
    for o in 5 6 7; do DXRPT_KERNEL_LIB_DIR=ab/t3 $T $cfg --label t3_tail$o --opt TAIL_OCCUPANCY=$o || exit 1; done
  done 2>&1 | grep -v amdgpu.ids
done
