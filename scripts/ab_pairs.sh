#!/bin/bash
# r03: shadow-ray pairs (DXRPT_SHADOW_PAIRS: ab/pairs2 tails + k_path, ab/pairs1 tails only, in-tree lib
# off): parity of the pairs2 build first, then ms/frame of the three builds, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
DXRPT_KERNEL_LIB_DIR=ab/pairs2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shipped.py -m gpu -q -x -rf \
    -k "split_is_bit_identical or megakernel_is_bit_identical or metric_frame or suntemple_1080p or 720p or spot or furnace or 4k" \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_pairs.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_pairs.log | tail -8
[ $rc -ne 0 ] && exit $rc
for cfg in "--config metric" "--config c4" "--config c3" "--config c2" "--config c5 --share 8 --rank 3" "--config metric --share 8 --rank 2"; do
  for b in dxrpathtracer_amd/lib ab/pairs1 ab/pairs2; do
    DXRPT_KERNEL_LIB_DIR=$b timeout -k 10 200 python -u scripts/time_frames.py --rounds 3 --frames 32 $cfg --label $b 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
