#!/bin/bash
# r03: three frames in flight (DXRPT_OPT_FRAME_OVERLAP 2) against two (1); XCD runs on the split schedule.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_steady_state.py -k "bit_identical" -m gpu -q -x -rf \
    --timeout 300 --timeout-method thread > gpurun_out/pytest_overlap3.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_overlap3.log | tail -5
[ $rc -ne 0 ] && exit $rc
T="timeout -k 10 200 python -u scripts/time_frames.py --rounds 3 --frames 48"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for cfg in "--config metric --share 8 --rank 2" "--config metric --share 8 --rank 6" "--config metric --share 4 --rank 1" \
           "--config metric --share 2 --rank 1" "--config metric" "--config c2" "--config c5 --share 8 --rank 5"; do
  run $cfg --overlap 1 --label ovl1
  run $cfg --overlap 2 --label ovl2
done
for cfg in "--config metric" "--config c4" "--config c5 --share 8 --rank 3"; do
  for x in 0 4 16; do run $cfg --xcd-chunk $x --label xcd$x; done
done
