#!/bin/bash
# r04 A/B: the SBVH / collapse parameters re-swept with the treelet pass on (runtime build options, in-tree
# build): triangle-test cost 1.25 / 1.5 (shipped) / 2.0 node visits, spatial-split budget 150 % (shipped) / 200 %.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import torch; torch.zeros(1, device='cuda')" || exit 1
T="timeout -k 10 150 python -u scripts/time_frames.py --rounds 3"
for cfg in "--config metric" "--config c2" "--config c3 --frames 16" "--config c4" "--config metric --share 8 --rank 2"; do
  for r in 1 2; do
    for o in "LEAF_COST=150" "LEAF_COST=125" "LEAF_COST=200" "SPATIAL_SPLITS=200"; do
      $T $cfg --opt $o --label $o 2>> gpurun_out/ab_build_params.err
      rc=$?; [ $rc -ne 0 ] && { echo "$o $cfg rc=$rc"; [ $rc -gt 1 ] && exit $rc; }
    done
  done
done
exit 0
