#!/bin/bash
# r05: sun-occluder cache in the chained last-depth shadow loop (ab/occ, -DDXRPT_OCC_CACHE=1): a path's
# last-depth sun ray first tests the triangle record that occluded it in an earlier frame; a hit decides it
# exactly (any occluder), a miss traverses as before.  Parity smoke first, then timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
DXRPT_KERNEL_LIB_DIR=ab/occ timeout -k 10 600 python -u -m pytest tests/test_gpu_steady_state.py -m gpu -q -x --timeout 300 --timeout-method thread -k "metric_1080p or overlapped_frames_are or band_share" > gpurun_out/pytest_occ.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_occ.log; [ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for cfg in metric c2 c4 c3; do
    run --label now --config $cfg
    DXRPT_KERNEL_LIB_DIR=ab/occ run --label occ --config $cfg
  done
  for rk in 2 5; do
    run --label now --share 8 --rank $rk --cur-copy
    DXRPT_KERNEL_LIB_DIR=ab/occ run --label occ --share 8 --rank $rk --cur-copy
  done
done
