#!/bin/bash
# r03: every rank's 1/8 share with alpha-tested triangles kept whole at the default budget / triangle cost.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 240 python -u scripts/time_frames.py --rounds 3 --frames 32"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for opt in "--label default" "--split-alpha 0 --label whole150"; do
  for r in 0 1 2 3 4 5 6 7; do run --config metric --share 8 --rank $r $opt; done
  run --config metric --share 4 --rank 1 $opt
  run --config metric --share 2 --rank 1 $opt
  run --config c5 --share 8 --rank 5 $opt
done
