#!/bin/bash
# r05: the texel decode table by LDS DMA, no barrier (ab/lutdma, -DDXRPT_LUT_DMA=1): parity through the
# variant (textured scenes on every schedule), then timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
DXRPT_KERNEL_LIB_DIR=ab/lutdma2 timeout -k 10 900 python -u -m pytest tests/test_gpu_steady_state.py tests/test_gpu_shipped.py tests/test_gpu_shipped_toggles.py tests/test_gpu_bake.py tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_lutdma.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_lutdma.log; [ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for cfg in metric c2 c4 c3; do
    run --label now --config $cfg
    DXRPT_KERNEL_LIB_DIR=ab/lutdma2 run --label lutdma2 --config $cfg
    DXRPT_KERNEL_LIB_DIR=ab/lutdma run --label lutdma --config $cfg
  done
  for rk in 2 5; do
    run --label now --share 8 --rank $rk --cur-copy
    DXRPT_KERNEL_LIB_DIR=ab/lutdma2 run --label lutdma2 --share 8 --rank $rk --cur-copy
  done
  run --label now --share 4 --rank 2 --cur-copy
  DXRPT_KERNEL_LIB_DIR=ab/lutdma2 run --label lutdma2 --share 4 --rank 2 --cur-copy
done
