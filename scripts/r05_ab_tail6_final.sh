#!/bin/bash
# r05 late: tail budget 6 vs 7 on the final kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for cfg in metric c4 c2 c3; do
    run --label default --config $cfg
    run --label tail6 --config $cfg --opt TAIL_OCCUPANCY=6
  done
done
