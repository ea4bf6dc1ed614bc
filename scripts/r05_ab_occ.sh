#!/bin/bash
# r05: register budgets of the split schedule on the r05 kernels (chained shadows, 115 % budget):
# tail 7 (default) vs 6 / 5 waves/SIMD, head 5 (default) vs 6 / 4, same box, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 120 python -u scripts/time_frames.py --rounds 5 "$@" || exit $?; }
for r in 1 2; do
  for cfg in metric c4 c3; do
    run --label base --config $cfg
    run --label tail6 --config $cfg --opt TAIL_OCCUPANCY=6
    run --label tail5 --config $cfg --opt TAIL_OCCUPANCY=5
    run --label head6 --config $cfg --opt MEGAKERNEL_OCCUPANCY=6 --opt TAIL_OCCUPANCY=7
    run --label head4 --config $cfg --opt MEGAKERNEL_OCCUPANCY=4 --opt TAIL_OCCUPANCY=7
  done
done
