#!/bin/bash
# r05: the spatial-split reference budget on the r05 builder (per-subtree allowance): 150 (r04 default) vs
# 110 / 115 / 125 / 135 %, same box, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 120 python -u scripts/time_frames.py --rounds 5 "$@" || exit $?; }
for r in 1 2; do
  for cfg in metric c4 c3 c2; do
    for b in 150 110 115 125 135; do run --label budget$b --config $cfg --opt SPATIAL_SPLITS=$b; done
  done
  for rk in 2 5 7; do for b in 150 110 115 125 135; do run --label budget$b --share 8 --rank $rk --opt SPATIAL_SPLITS=$b; done; done
done
