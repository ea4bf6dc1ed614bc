#!/bin/bash
# r04 A/B: spatial-split budget 150 % (shipped) against 175 % on the metric, its slowest 1/8 shares and C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import torch; torch.zeros(1, device='cuda')" || exit 1
T="timeout -k 10 150 python -u scripts/time_frames.py --rounds 3"
for cfg in "--config metric" "--config c4" "--config metric --share 8 --rank 1" "--config metric --share 8 --rank 2"; do
  for r in 1 2; do
    for o in "SPATIAL_SPLITS=150" "SPATIAL_SPLITS=175"; do
      $T $cfg --opt $o --label $o 2>> gpurun_out/ab_split175.err
      rc=$?; [ $rc -ne 0 ] && { echo "$o $cfg rc=$rc"; [ $rc -gt 1 ] && exit $rc; }
    done
  done
done
exit 0
