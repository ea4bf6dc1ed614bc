#!/bin/bash
# r05: the head's depth-1 sun shadow ray kept in registers for the packet traversal (ab/sunregs,
# -DDXRPT_HEAD_SUN_REGS=1; the slot's contribution still loaded, consumed after the traversal).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
DXRPT_KERNEL_LIB_DIR=ab/sunregs timeout -k 10 900 python -u -m pytest tests/test_gpu_steady_state.py tests/test_gpu_shipped.py tests/test_gpu_shipped_toggles.py tests/test_gpu_parity.py -k "split or metric or shipped or toggles or overlapped or band_share or c5 or c3 or suntemple or 720p or megakernel" -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_sunregs.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_sunregs.log; [ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for cfg in metric c2 c4 c3; do
    run --label now --config $cfg
    DXRPT_KERNEL_LIB_DIR=ab/sunregs run --label sunregs --config $cfg
  done
  run --label now --share 2 --rank 0 --cur-copy
  DXRPT_KERNEL_LIB_DIR=ab/sunregs run --label sunregs --share 2 --rank 0 --cur-copy
done
