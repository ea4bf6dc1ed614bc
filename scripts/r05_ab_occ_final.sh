#!/bin/bash
# r05 late: head budget re-swept on the final kernels (LDS-DMA table: head<6> spills 34 -> 19).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for cfg in metric c4 c2; do
    run --label default --config $cfg
    for h in 5 6 7; do run --label head$h --config $cfg --opt MEGAKERNEL_OCCUPANCY=$h --opt TAIL_OCCUPANCY=7; done
  done
  run --label default --share 2 --rank 0 --cur-copy
  run --label head6 --share 2 --rank 0 --cur-copy --opt MEGAKERNEL_OCCUPANCY=6 --opt TAIL_OCCUPANCY=7
done
