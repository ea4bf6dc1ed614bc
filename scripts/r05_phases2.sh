#!/bin/bash
# r05 late: per-phase lane time of the head and tails with packed / inlined material maps (ab/phases,
# -DDXRPT_DIAG_PHASES=1), frame-at-a-time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for cfg in metric c3 c4; do
  DXRPT_KERNEL_LIB_DIR=ab/phases timeout -k 10 120 python -u scripts/time_frames.py --label phases --config $cfg --rounds 3 --phases --opt FRAME_OVERLAP=0 2>&1 | grep -v amdgpu.ids || exit 1
done
