#!/bin/bash
# r05: LDS-DMA table fill everywhere but the non-last split tails (default) vs in those too (ab/dmaall).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for cfg in c3 metric c5; do
    run --label default --config $cfg
    DXRPT_KERNEL_LIB_DIR=ab/dmaall run --label dmaall --config $cfg
  done
done
