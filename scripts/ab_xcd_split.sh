#!/bin/bash
# r03: XCD runs (DXRPT_OPT_XCD_CHUNK) on the split schedule's head and tails under overlapped frames.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 200 python -u scripts/time_frames.py --rounds 3 --frames 32"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for cfg in "--config metric" "--config c4" "--config c5 --share 8 --rank 3" "--config c3"; do
  for x in 8 0 4 16 32; do run $cfg --xcd-chunk $x --label xcd$x; done
done
