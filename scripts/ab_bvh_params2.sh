#!/bin/bash
# r03: SBVH reference budget x triangle cost sweep under the final schedule, every 1-GPU config.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 240 python -u scripts/time_frames.py --rounds 3 --frames 24"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for cfg in "--config metric" "--config c4" "--config c5 --share 8 --rank 3" "--config c2" "--config c3"; do
  run $cfg --label default
  for sp in 200 250 300; do run $cfg --spatial $sp --leaf-cost 125 --label s${sp}l125; done
  run $cfg --spatial 250 --label s250l150
done
