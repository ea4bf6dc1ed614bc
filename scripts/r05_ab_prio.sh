#!/bin/bash
# r05: issue priority (s_setprio) for the costliest waves of cost-ordered frames (the 1/8 shares), whose
# one round of waves ends with the slowest few alone on the chip (scripts/wave_clocks.py --ordered):
# ab/prio1 top 1/32 of the waves at priority 3, prio2 top 1/8, prio3 graded 3/2/1 over the top 1/32, 1/8, 1/4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 120 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for rk in 1 2 4 7; do
    run --label base --share 8 --rank $rk
    for v in 1 2 3; do DXRPT_KERNEL_LIB_DIR=ab/prio$v run --label prio$v --share 8 --rank $rk; done
  done
done
