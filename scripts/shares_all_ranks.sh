#!/bin/bash
# Every rank's band share of the metric frame at N = 8, 4, 2 (and C5's 1/8 shares), default schedule, one
# MI355X: the projected N-GPU frame time is the slowest rank's (plus the gather; N>1 runs are the driver's).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 200 python -u scripts/time_frames.py --rounds 3 --frames 32 ${SHARE_FLAGS:-}"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
run --config metric --label default
for n in 8 4 2; do
  for ((r = 0; r < n; r++)); do run --config metric --share $n --rank $r --label default; done
done
for ((r = 0; r < 8; r++)); do run --config c5 --share 8 --rank $r --label default; done
