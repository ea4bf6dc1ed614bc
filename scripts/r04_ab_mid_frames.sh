#!/bin/bash
# r04 A/B: mid-size frames (C2 720p, the metric's 1/4 share) that run the single k_path at 6-7 waves/SIMD (octant
# child order, spills) against the depth-split schedule and k_path at 5 waves/SIMD (nearest-child-first closest
# hits, near-to-far packet shadows), after the r04 traversal-order changes.  Runtime options, in-tree build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import torch; torch.zeros(1, device='cuda')" || exit 1
T="timeout -k 10 150 python -u scripts/time_frames.py --rounds 3"
for cfg in "--config c2" "--config metric --share 4 --rank 1" "--config metric --share 4 --rank 2"; do
  for r in 1 2; do
    for o in "FRAME_OVERLAP=1" "MEGAKERNEL_SPLIT=1" "MEGAKERNEL_OCCUPANCY=5" "MEGAKERNEL_OCCUPANCY=6"; do
      $T $cfg --opt $o --label $o 2>> gpurun_out/ab_mid_frames.err
      rc=$?; [ $rc -ne 0 ] && { echo "$o $cfg rc=$rc"; [ $rc -gt 1 ] && exit $rc; }
    done
  done
done
exit 0
