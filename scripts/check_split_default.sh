#!/bin/bash
# r03: GPU parity of the shipped / steady-state schedules after the split-default change, then the
# default's ms/frame on every config and the busiest shares.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_shipped.py tests/test_gpu_steady_state.py -m gpu -q -x -rf \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_split.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_split.log | tail -8
[ $rc -ne 0 ] && exit $rc
T="timeout -k 10 200 python -u scripts/time_frames.py --rounds 3 --frames 32"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for c in metric c4 c2 c3 c5; do run --config $c --label default; done
run --config c5 --share 8 --rank 3 --label default
run --config metric --share 2 --rank 1 --label default
run --config metric --occ 7 --label head7
run --config c4 --occ 7 --label head7
run --config c5 --share 8 --rank 3 --occ 7 --label head7
run --config c3 --occ 7 --label head7
