#!/bin/bash
# r04 A/B: the SBVH spatial-split budget (150 % shipped at the time / 200 / 250 / 300 % of the triangles) and treelet
# passes (1 / 2) after the traversal-order changes.  Runtime build options, in-tree build, two interleaved passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import torch; torch.zeros(1, device='cuda')" || exit 1
T="timeout -k 10 150 python -u scripts/time_frames.py --rounds 3"
for cfg in "--config metric" "--config c2" "--config c3 --frames 16" "--config c4" "--config c5 --frames 8" "--config metric --share 8 --rank 2"; do
  for r in 1 2; do
    for o in "SPATIAL_SPLITS=150" "SPATIAL_SPLITS=200" "SPATIAL_SPLITS=250" "SPATIAL_SPLITS=300"; do
      $T $cfg --opt $o --label $o 2>> gpurun_out/ab_split_budget.err
      rc=$?; [ $rc -ne 0 ] && { echo "$o $cfg rc=$rc"; [ $rc -gt 1 ] && exit $rc; }
    done
    $T $cfg --opt SPATIAL_SPLITS=200 --opt TREELET_PASSES=2 --label S200_T2 2>> gpurun_out/ab_split_budget.err
  done
done
exit 0
