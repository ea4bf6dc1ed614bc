#!/bin/bash
# A/B of kernel builds on the GPU box: each directory in $BUILDS (default: every ab/*/ holding a
# libdxrpt.so, plus the in-tree lib) is timed by scripts/time_frames.py in its own process, the
# builds interleaved for $ROUNDS rounds.  Extra arguments go to time_frames.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BUILDS=${BUILDS:-"dxrpathtracer_amd/lib $(ls -d ab/*/ 2>/dev/null | tr '\n' ' ')"}
for r in $(seq 1 ${ROUNDS:-2}); do
  for b in $BUILDS; do
    DXRPT_KERNEL_LIB_DIR=$b timeout -k 10 120 python -u scripts/time_frames.py --label "$b" "$@" || exit $?
  done
done
