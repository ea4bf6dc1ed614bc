#!/bin/bash
# r03: SBVH budget with alpha-tested triangles kept whole (DXRPT_OPT_SPLIT_ALPHA 0), every 1-GPU config;
# bit-identity of the alpha paths first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 240 python -u scripts/time_frames.py --rounds 3 --frames 24"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for cfg in "--config c4" "--config metric" "--config c5 --share 8 --rank 3" "--config c2" "--config c3"; do
  run $cfg --label default
  run $cfg --split-alpha 0 --label whole150
  run $cfg --spatial 200 --leaf-cost 125 --split-alpha 0 --label whole200l125
  run $cfg --spatial 300 --leaf-cost 125 --split-alpha 0 --label whole300l125
done
