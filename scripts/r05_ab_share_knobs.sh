#!/bin/bash
# r05: the band shares' schedule knobs re-swept with three frames in flight (and the per-frame snapshot on
# the render stream, as NativeGather runs it): occupancy, cost-ordered waves, the split schedule.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 --cur-copy "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for rk in 1 2; do
    run --label default --share 8 --rank $rk
    for o in 5 6 7; do run --label occ$o --share 8 --rank $rk --opt MEGAKERNEL_OCCUPANCY=$o; done
    run --label order0 --share 8 --rank $rk --opt WAVE_ORDER=0
    run --label split --share 8 --rank $rk --opt MEGAKERNEL_SPLIT=1
  done
  run --label default --share 4 --rank 2
  for o in 4 6 7; do run --label occ$o --share 4 --rank 2 --opt MEGAKERNEL_OCCUPANCY=$o; done
  run --label order1 --share 4 --rank 2 --opt WAVE_ORDER=1
  run --label split --share 4 --rank 2 --opt MEGAKERNEL_SPLIT=1
  run --label default --share 2 --rank 0
  run --label nosplit --share 2 --rank 0 --opt MEGAKERNEL_SPLIT=0
  run --label default --config c2
  run --label ovl2 --config c2 --opt FRAME_OVERLAP=2
  run --label split --config c2 --opt FRAME_OVERLAP=2 --opt MEGAKERNEL_SPLIT=1
done
