#!/bin/bash
# r05: the BVH build parameters re-swept on the r05 builder and kernels (same box, interleaved):
# defaults (1 treelet pass, leaf cost 1.5, budget 150 %) vs 2 treelet passes, leaf cost 1.25 / 2.0,
# budget 125 %.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 120 python -u scripts/time_frames.py --rounds 5 "$@" || exit $?; }
for r in 1 2; do
  for cfg in metric c4 c3; do
    run --label default --config $cfg
    run --label treelet2 --config $cfg --opt TREELET_PASSES=2
    run --label leaf125 --config $cfg --opt LEAF_COST=125
    run --label leaf200 --config $cfg --opt LEAF_COST=200
    run --label budget125 --config $cfg --opt SPATIAL_SPLITS=125
  done
  for rk in 2 5; do
    run --label default --share 8 --rank $rk
    run --label treelet2 --share 8 --rank $rk --opt TREELET_PASSES=2
    run --label leaf125 --share 8 --rank $rk --opt LEAF_COST=125
    run --label leaf200 --share 8 --rank $rk --opt LEAF_COST=200
    run --label budget125 --share 8 --rank $rk --opt SPATIAL_SPLITS=125
  done
done
