#!/bin/bash
# r04 A/B, second part: spatial-split budget 150 % against 175 % on every rank of the 1/8 share and on C2 / C3 / C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import torch; torch.zeros(1, device='cuda')" || exit 1
T="timeout -k 10 150 python -u scripts/time_frames.py --rounds 3"
for cfg in "--config c2" "--config c3 --frames 16" "--config c5 --frames 8" "--config metric --share 8 --rank 0" "--config metric --share 8 --rank 3" "--config metric --share 8 --rank 4" "--config metric --share 8 --rank 5" "--config metric --share 8 --rank 6" "--config metric --share 8 --rank 7" "--config metric --share 4 --rank 1"; do
  for o in "SPATIAL_SPLITS=150" "SPATIAL_SPLITS=175"; do
    $T $cfg --opt $o --label $o 2>> gpurun_out/ab_split175.err
    rc=$?; [ $rc -ne 0 ] && { echo "$o $cfg rc=$rc"; [ $rc -gt 1 ] && exit $rc; }
  done
done
exit 0
