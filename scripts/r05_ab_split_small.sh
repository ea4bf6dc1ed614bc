#!/bin/bash
# r05 late: the split schedule on the band shares now that its depth-2 queue is direct-mapped (no
# returning atomic in the head): 1/4 and 1/8 shares split vs the default k_path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 --cur-copy "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for rk in 1 2; do
    run --label default --share 4 --rank $rk
    run --label split --share 4 --rank $rk --opt MEGAKERNEL_SPLIT=1
  done
  run --label default --share 8 --rank 2
  run --label split --share 8 --rank 2 --opt MEGAKERNEL_SPLIT=1
  run --label split-h4 --share 8 --rank 2 --opt MEGAKERNEL_SPLIT=1 --opt MEGAKERNEL_OCCUPANCY=4 --opt TAIL_OCCUPANCY=7
done
