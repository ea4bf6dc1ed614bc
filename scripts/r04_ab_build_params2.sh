#!/bin/bash
# r04 A/B: the build options re-swept after the traversal-order changes (far-to-near any-hit, nearest-first closest
# hits): treelet passes 0 / 1 (shipped) / 2, spatial-split budget 200 %, triangle-test cost 1.25 / 2.0.  Runtime
# options, in-tree build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import torch; torch.zeros(1, device='cuda')" || exit 1
T="timeout -k 10 150 python -u scripts/time_frames.py --rounds 3"
for cfg in "--config metric" "--config c3 --frames 16" "--config c4" "--config metric --share 8 --rank 2"; do
  for r in 1 2; do
    for o in "TREELET_PASSES=1" "TREELET_PASSES=0" "TREELET_PASSES=2" "SPATIAL_SPLITS=200" "LEAF_COST=125" "LEAF_COST=200"; do
      $T $cfg --opt $o --label $o 2>> gpurun_out/ab_build_params2.err
      rc=$?; [ $rc -ne 0 ] && { echo "$o $cfg rc=$rc"; [ $rc -gt 1 ] && exit $rc; }
    done
  done
done
exit 0
