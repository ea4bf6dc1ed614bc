#!/bin/bash
# r05: head 6 above 1.5M paths -- shipped-schedule parity tests, then metric / C3 / C4 against head 5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_shipped_toggles.py tests/test_gpu_shipped.py tests/test_gpu_steady_state.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_head6.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_head6.log; [ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for cfg in metric c3 c4; do
    run --label default --config $cfg
    run --label head5 --config $cfg --opt MEGAKERNEL_OCCUPANCY=5 --opt TAIL_OCCUPANCY=7
  done
done
