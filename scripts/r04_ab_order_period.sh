#!/bin/bash
# r04 A/B: the 1/8 share's cost-order refresh period (DXRPT_OPT_WAVE_ORDER_PERIOD 16 shipped / 4 / 1) on its slowest ranks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import torch; torch.zeros(1, device='cuda')" || exit 1
T="timeout -k 10 150 python -u scripts/time_frames.py --rounds 3"
for rk in 1 2 4; do
  for r in 1 2; do
    for o in ${PERIODS:-"WAVE_ORDER_PERIOD=16" "WAVE_ORDER_PERIOD=4" "WAVE_ORDER_PERIOD=1"}; do
      $T --config metric --share 8 --rank $rk --opt $o --label $o 2>> gpurun_out/ab_order_period.err
      rc=$?; [ $rc -ne 0 ] && { echo "$o rank $rk rc=$rc"; [ $rc -gt 1 ] && exit $rc; }
    done
  done
done
exit 0
