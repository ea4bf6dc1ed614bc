#!/bin/bash
# r05: the tails' material taps in the grouped (branch-free, four loads together) form now that packed /
# inlined maps leave two taps per hit (ab/tailgrp, -DDXRPT_TAIL_GROUPED_TAPS=1) vs per-texel (default).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for cfg in metric c2 c4 c3; do
    run --label now --config $cfg
    DXRPT_KERNEL_LIB_DIR=ab/tailgrp run --label tailgrp --config $cfg
  done
done
