#!/bin/bash
# r03: parity of the split schedule with closest-hit triangle pairs in the tails, then its budgets.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_shipped.py tests/test_gpu_steady_state.py tests/test_gpu_parity.py \
    -k "shipped or steady or split or 4k or L8 or metric or suntemple" -m gpu -q -x -rf --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_tail_pairs.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_tail_pairs.log | tail -5
[ $rc -ne 0 ] && exit $rc
T="timeout -k 10 200 python -u scripts/time_frames.py --rounds 3 --frames 32"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for cfg in "--config metric" "--config c4" "--config c5 --share 8 --rank 3"; do
  run $cfg --label default
  run $cfg --tail-occ 6 --label tail6
done
run --config c5 --label default
# k_path (C2, the band shares) with per-lane triangle pairs too (ab/mch1: DXRPT_MEGA_PIPE_CH 1)
for cfg in "--config c2" "--config metric --share 8 --rank 2" "--config metric --share 4 --rank 1" "--config metric --share 2 --rank 1"; do
  for b in dxrpathtracer_amd/lib ab/mch1; do
    DXRPT_KERNEL_LIB_DIR=$b $T $cfg --label $b 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
