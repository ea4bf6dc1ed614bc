#!/bin/bash
# r03: the split head's packet traversals with leaf triangles two at a time (ab/hp1 closest hit, ab/hp2
# depth-1 sun shadows, ab/hp3 both): parity of hp3 on the shipped frames, then ms/frame.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
DXRPT_KERNEL_LIB_DIR=ab/hp3 timeout -k 10 300 python -u -m pytest tests/test_gpu_shipped.py -k "metric or suntemple" -m gpu -q -x -rf \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_hp3.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_hp3.log | tail -3
[ $rc -ne 0 ] && exit $rc
for cfg in "--config metric" "--config c4" "--config c5 --share 8 --rank 3" "--config c3"; do
  for b in dxrpathtracer_amd/lib ab/hp1 ab/hp2 ab/hp3; do
    DXRPT_KERNEL_LIB_DIR=$b timeout -k 10 240 python -u scripts/time_frames.py --rounds 3 --frames 24 $cfg --label $b 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
