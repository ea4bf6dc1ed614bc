#!/bin/bash
# r05: the split schedule's tails at 8 waves/SIMD (64 registers, more spills) vs 7 (default).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 120 python -u scripts/time_frames.py --rounds 5 "$@" || exit $?; }
for r in 1 2; do
  for cfg in metric c4 c3 c2; do
    run --label base --config $cfg
    run --label tail8 --config $cfg --opt TAIL_OCCUPANCY=8
  done
  for rk in 2 5; do run --label base --share 8 --rank $rk; run --label tail8 --share 8 --rank $rk --opt TAIL_OCCUPANCY=8; done
done
