#!/bin/bash
# r05: frames in flight (DXRPT_OPT_FRAME_OVERLAP n: n + 1 frames) -- 2 (default) vs 3 vs 4 -- on the
# band shares (one round of waves, latency-bound: wave_clocks busy 0.22-0.27) and the full frames.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 120 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for o in 1 2 3; do
    for rk in 2 7; do run --label ovl$o --share 8 --rank $rk --opt FRAME_OVERLAP=$o; done
    run --label ovl$o --share 4 --rank 2 --opt FRAME_OVERLAP=$o
    run --label ovl$o --share 2 --rank 0 --opt FRAME_OVERLAP=$o
    run --label ovl$o --config metric --opt FRAME_OVERLAP=$o
    run --label ovl$o --config c2 --opt FRAME_OVERLAP=$o
  done
done
