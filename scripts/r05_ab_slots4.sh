#!/bin/bash
# r05: four frames in flight (ab/slots4, -DDXRPT_OVERLAP_SLOTS=4) against three, with 8 hardware queues
# (what bench.py gives multi-GPU ranks) and the per-frame snapshot on the render stream.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 --cur-copy "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for rk in 2 7; do
    run --label slots3 --share 8 --rank $rk
    DXRPT_KERNEL_LIB_DIR=ab/slots4 run --label slots4 --share 8 --rank $rk
  done
  run --label slots3 --share 4 --rank 2
  DXRPT_KERNEL_LIB_DIR=ab/slots4 run --label slots4 --share 4 --rank 2
  run --label slots3 --share 2 --rank 0
  DXRPT_KERNEL_LIB_DIR=ab/slots4 run --label slots4 --share 2 --rank 0
  run --label slots3 --config metric
  DXRPT_KERNEL_LIB_DIR=ab/slots4 run --label slots4 --config metric
done
