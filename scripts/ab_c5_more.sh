#!/bin/bash
# r03: C5 (4K L=6, one GPU) budgets and parts under overlapped frames, same box; then the host cost of
# the bench loop per frame (scripts/host_overhead.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 200 python -u scripts/time_frames.py --rounds 3 --frames 24"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  run --config c5 --label default
  run --config c5 --parts 2 --label parts2
  run --config c5 --tail-occ 8 --label tail8
  run --config c5 --occ 6 --tail-occ 7 --label head6
done
timeout -k 10 200 python -u scripts/host_overhead.py 2>&1 | grep -v amdgpu.ids
