#!/bin/bash
# r05 late: the cost order's rebuild period (default 64 frames) on the 1/8 shares with three frames in flight.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 --cur-copy "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for rk in 1 2; do
    run --label default --share 8 --rank $rk
    for p in 16 256; do run --label period$p --share 8 --rank $rk --opt WAVE_ORDER_PERIOD=$p; done
  done
done
