#!/bin/bash
# A/B of the depth-split megakernel (DXRPT_OPT_MEGAKERNEL_SPLIT) against the single k_path on the
# BASELINE configs; each line from scripts/time_frames.py.  Extra env: CONFIGS, OCCS ("head:tail ...").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 180 python -u scripts/time_frames.py --rounds ${ROUNDS:-3} --frames ${FRAMES:-24}"
for c in ${CONFIGS:-metric c3 c4 c5 c2}; do
  $T --config $c --msplit 0 --label single 2>&1 | grep -v amdgpu.ids || exit 1
  for o in ${OCCS:-7:7 6:6 5:6 5:5 6:7}; do
    $T --config $c --msplit 1 --occ ${o%%:*} --tail-occ ${o##*:} --label split 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
