#!/bin/bash
# r04 A/B: the metric's 1/2 share (1.04M paths, the depth-split schedule by size) against the single k_path at 7 (octant
# order) and 5 waves/SIMD (nearest-first) after the traversal-order changes.  Runtime options, two passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import torch; torch.zeros(1, device='cuda')" || exit 1
T="timeout -k 10 150 python -u scripts/time_frames.py --rounds 3"
for rk in 0 1; do
  for r in 1 2; do
    for o in "FRAME_OVERLAP=1" "MEGAKERNEL_SPLIT=0" "MEGAKERNEL_SPLIT=0 --opt MEGAKERNEL_OCCUPANCY=5"; do
      $T --config metric --share 2 --rank $rk --opt $o --label "$o" 2>> gpurun_out/ab_half_share.err
      rc=$?; [ $rc -ne 0 ] && { echo "$o rank $rk rc=$rc"; [ $rc -gt 1 ] && exit $rc; }
    done
  done
done
exit 0
