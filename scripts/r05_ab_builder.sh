#!/bin/bash
# r05: the parallel SBVH builder (per-subtree duplication budget, degenerate-centroid splits within the
# budget) against r04's serial builder (ab/r04: the r04 library, built from c702763), same box, interleaved;
# then the new builder's spatial-split budget 150 / 175 / 200 % (item 6 of the r04 verdict).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 120 python -u scripts/time_frames.py --rounds 5 "$@" || exit $?; }
for r in 1 2; do
  for cfg in metric c4 c3 c2; do
    for b in ab/r04 dxrpathtracer_amd/lib; do DXRPT_KERNEL_LIB_DIR=$b run --label $b --config $cfg; done
  done
  for rk in 2 5; do
    for b in ab/r04 dxrpathtracer_amd/lib; do DXRPT_KERNEL_LIB_DIR=$b run --label $b --share 8 --rank $rk; done
  done
done
for cfg in metric c4; do
  for sp in 175 200; do run --label "budget$sp" --config $cfg --opt SPATIAL_SPLITS=$sp; done
done
for rk in 2 5; do for sp in 175 200; do run --label "budget$sp" --share 8 --rank $rk --opt SPATIAL_SPLITS=$sp; done; done
