#!/bin/bash
# r03: BVH8 build parameters under the final schedule (triangle cost in the SAH-DP collapse, SBVH budget).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 240 python -u scripts/time_frames.py --rounds 3 --frames 32"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for cfg in "--config metric" "--config c4" "--config c5 --share 8 --rank 3"; do
  run $cfg --label default
  for lc in 100 125 200; do run $cfg --leaf-cost $lc --label leaf$lc; done
  for sp in 120 200; do run $cfg --spatial $sp --label sbvh$sp; done
done
