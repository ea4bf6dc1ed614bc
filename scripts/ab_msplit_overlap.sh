#!/bin/bash
# r03: the depth-split schedule on short-path frames once frames overlap (metric, C4, C2, shares).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 200 python -u scripts/time_frames.py --rounds 3 --frames 32"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for c in metric c4 c2; do
  run --config $c --label default
  run --config $c --msplit 1 --parts 1 --label split1
  run --config $c --msplit 1 --parts 2 --label split2
  run --config $c --msplit 1 --parts 2 --occ 7 --label split2o7
done
run --config metric --share 2 --rank 1 --label default
run --config metric --share 2 --rank 1 --msplit 1 --parts 2 --label split2
run --config metric --share 4 --rank 1 --label default
run --config metric --share 4 --rank 1 --msplit 1 --parts 2 --label split2
run --config c5 --msplit 1 --parts 2 --label split2
run --config c5 --share 8 --rank 3 --label default
run --config c5 --share 8 --rank 3 --msplit 1 --parts 2 --label split2
