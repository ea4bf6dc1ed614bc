#!/bin/bash
# r04 A/B: the split schedule's register budgets re-checked after the traversal-order changes: head 4 / 5 (shipped) /
# 6 waves/SIMD (DXRPT_OPT_MEGAKERNEL_OCCUPANCY), tail 6 / 7 (shipped) (DXRPT_OPT_TAIL_OCCUPANCY).  Runtime options.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import torch; torch.zeros(1, device='cuda')" || exit 1
T="timeout -k 10 150 python -u scripts/time_frames.py --rounds 3"
for cfg in "--config metric" "--config c3 --frames 16" "--config c4" "--config c5 --frames 8"; do
  for r in 1 2; do
    for o in "TAIL_OCCUPANCY=7" "TAIL_OCCUPANCY=6" "MEGAKERNEL_OCCUPANCY=4 --opt TAIL_OCCUPANCY=7" "MEGAKERNEL_OCCUPANCY=6 --opt TAIL_OCCUPANCY=7"; do
      $T $cfg --opt $o --label "head/tail $o" 2>> gpurun_out/ab_budgets.err
      rc=$?; [ $rc -ne 0 ] && { echo "$o $cfg rc=$rc"; [ $rc -gt 1 ] && exit $rc; }
    done
  done
done
exit 0
