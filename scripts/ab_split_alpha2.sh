#!/bin/bash
# r03: SBVH budget / triangle cost around 200 % / 1.25 with alpha-tested triangles kept whole.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 240 python -u scripts/time_frames.py --rounds 3 --frames 24"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for cfg in "--config c4" "--config metric" "--config c5 --share 8 --rank 3" "--config metric --share 8 --rank 2"; do
  run $cfg --split-alpha 0 --spatial 200 --leaf-cost 125 --label w200l125
  run $cfg --split-alpha 0 --spatial 175 --leaf-cost 125 --label w175l125
  run $cfg --split-alpha 0 --spatial 200 --leaf-cost 150 --label w200l150
  run $cfg --split-alpha 0 --spatial 200 --leaf-cost 100 --label w200l100
  run $cfg --split-alpha 0 --spatial 150 --leaf-cost 125 --label w150l125
done
