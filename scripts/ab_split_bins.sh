#!/bin/bash
# r03: direction-binned split queues (DXRPT_OPT_SPLIT_BINS) -- bit-identity, then ms/frame A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "split_is_bit_identical" -m gpu -q -x -rf \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_bins.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_bins.log | tail -8
[ $rc -ne 0 ] && exit $rc
T="timeout -k 10 200 python -u scripts/time_frames.py --rounds 3 --frames 32"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for c in metric c4 c3 c5; do
  run --config $c --label default
  run --config $c --bins 1 --label bins
done
run --config c5 --share 8 --rank 3 --label default
run --config c5 --share 8 --rank 3 --bins 1 --label bins
