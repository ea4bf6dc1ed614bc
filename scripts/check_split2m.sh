#!/bin/bash
# r03 final: parity with the 2M-vertex split threshold, then the 1/2 shares.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_shipped.py tests/test_gpu_steady_state.py -m gpu -q -x -rf \
    --timeout 300 --timeout-method thread > gpurun_out/pytest_split2m.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_split2m.log | tail -3
[ $rc -ne 0 ] && exit $rc
T="timeout -k 10 240 python -u scripts/time_frames.py --rounds 3 --frames 32"
for r in 0 1; do $T --config metric --share 2 --rank $r --label default 2>&1 | grep -v amdgpu.ids || exit 1; done
