#!/bin/bash
# r03: split-schedule register budgets under overlapped frames (head 5 = no spills, tail 6 = 6 spills).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 200 python -u scripts/time_frames.py --rounds 3 --frames 32"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for c in metric c4 c3; do
  run --config $c --label default
  run --config $c --occ 5 --tail-occ 7 --label h5t7
  run --config $c --occ 5 --tail-occ 6 --label h5t6
  run --config $c --occ 7 --tail-occ 6 --label h7t6
done
run --config c5 --share 8 --rank 3 --label default
run --config c5 --share 8 --rank 3 --occ 5 --tail-occ 7 --label h5t7
run --config c5 --label default
run --config c5 --occ 5 --tail-occ 7 --label h5t7
