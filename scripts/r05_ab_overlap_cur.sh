#!/bin/bash
# r05: 2 vs 3 frames in flight with the per-frame slab snapshot on the caller's stream (a gather without a
# side stream), default 4 hardware queues; shares and full frames.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for o in 1 2; do
    for rk in 0 1 2 3 4 5 6 7; do run --label ovl$o --share 8 --rank $rk --opt FRAME_OVERLAP=$o --cur-copy; done
    run --label ovl$o --share 4 --rank 2 --opt FRAME_OVERLAP=$o --cur-copy
    run --label ovl$o --share 2 --rank 0 --opt FRAME_OVERLAP=$o --cur-copy
    run --label ovl$o --config c5 --share 8 --rank 2 --opt FRAME_OVERLAP=$o --cur-copy
  done
done
