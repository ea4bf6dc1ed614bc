#!/bin/bash
# r05: the current build against the build before packed / inlined material taps (ab/head6 = commit
# 0c80b39), same box, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
bash scripts/r05_ab_slots4.sh
for r in 1 2; do
  for cfg in metric c2 c4; do
    run --label now --config $cfg
    run --label now-taps0 --config $cfg --opt PACKED_TAPS=0
    DXRPT_KERNEL_LIB_DIR=ab/head6 run --label head6 --config $cfg
  done
done
