#!/bin/bash
# A/B: overlapped frames on / off (DXRPT_OPT_FRAME_OVERLAP) on the single-kernel configs and band shares.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 200 python -u scripts/time_frames.py --rounds 3 --frames 24"
for r in 1 2; do
  for ovl in 0 1; do
    for args in "--config metric" "--config c4" "--config c2" "--config metric --share 8 --rank 5" "--config metric --share 8 --rank 2" "--config metric --share 4 --rank 1" "--config metric --share 2 --rank 1" "--config c5 --share 8 --rank 3"; do
      $T $args --overlap $ovl --label ovl$ovl 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done
