#!/bin/bash
# r03 final tree: head register budget 5 (96 VGPRs, no spills) / 6 / 7 (72, the default) with tails at 7.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 240 python -u scripts/time_frames.py --rounds 3 --frames 32"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for cfg in "--config metric" "--config c4" "--config c5 --share 8 --rank 3" "--config c3"; do
    run $cfg --label head7
    run $cfg --occ 5 --tail-occ 7 --label head5
    run $cfg --occ 6 --tail-occ 7 --label head6
  done
done
