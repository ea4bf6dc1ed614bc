#!/bin/bash
# r05: 2 vs 3 frames in flight with a NativeGather-like side stream per frame (the multi-GPU run's fifth
# stream: GPU_MAX_HW_QUEUES is 4), on the 1/8, 1/4 and 1/2 shares; then C3, C4, C5 full frames.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for o in 1 2; do
    run --label ovl$o --share 8 --rank 2 --opt FRAME_OVERLAP=$o --side-stream
    run --label ovl$o --share 8 --rank 5 --opt FRAME_OVERLAP=$o --side-stream
    run --label ovl$o --share 4 --rank 2 --opt FRAME_OVERLAP=$o --side-stream
    run --label ovl$o --share 2 --rank 0 --opt FRAME_OVERLAP=$o --side-stream
    run --label ovl$o --config c5 --share 8 --rank 2 --opt FRAME_OVERLAP=$o --side-stream
  done
done
for o in 1 2; do
  for cfg in c3 c4; do run --label ovl$o --config $cfg --opt FRAME_OVERLAP=$o; done
  run --label ovl$o --config c5 --rounds 3 --frames 16 --opt FRAME_OVERLAP=$o
done
