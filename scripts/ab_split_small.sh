#!/bin/bash
# r03 final: the depth-split schedule (head 5 / tail 7) on the frames below the 4M-vertex threshold.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 240 python -u scripts/time_frames.py --rounds 3 --frames 32"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for cfg in "--config c2" "--config metric --share 2 --rank 1" "--config c3 --share 8 --rank 3" "--config metric --share 4 --rank 1"; do
    run $cfg --label default
    run $cfg --msplit 1 --label split
  done
done
