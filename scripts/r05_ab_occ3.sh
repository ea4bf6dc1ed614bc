#!/bin/bash
# r05: the split schedule's register budgets re-swept with three frames in flight (head 5 / tail 7 default).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for cfg in metric c2 c4; do
    run --label h5t7 --config $cfg
    run --label h4t7 --config $cfg --opt MEGAKERNEL_OCCUPANCY=4 --opt TAIL_OCCUPANCY=7
    run --label h6t7 --config $cfg --opt MEGAKERNEL_OCCUPANCY=6 --opt TAIL_OCCUPANCY=7
    run --label h5t6 --config $cfg --opt MEGAKERNEL_OCCUPANCY=5 --opt TAIL_OCCUPANCY=6
  done
  run --label h5t7 --share 2 --rank 0 --cur-copy
  run --label h4t7 --share 2 --rank 0 --cur-copy --opt MEGAKERNEL_OCCUPANCY=4 --opt TAIL_OCCUPANCY=7
  run --label h6t7 --share 2 --rank 0 --cur-copy --opt MEGAKERNEL_OCCUPANCY=6 --opt TAIL_OCCUPANCY=7
  run --label h5t7 --config c5 --share 8 --rank 2 --cur-copy
  run --label h4t7 --config c5 --share 8 --rank 2 --cur-copy --opt MEGAKERNEL_OCCUPANCY=4 --opt TAIL_OCCUPANCY=7
  run --label h6t7 --config c5 --share 8 --rank 2 --cur-copy --opt MEGAKERNEL_OCCUPANCY=6 --opt TAIL_OCCUPANCY=7
done
