#!/bin/bash
# r05: packed / inlined material maps with the opacity tap kept plain, against the pre-packing build
# (ab/head6 = commit 0c80b39), same box, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for cfg in metric c2 c4 c3; do
    run --label now --config $cfg
    run --label now-packed1 --config $cfg --opt PACKED_TAPS=1
    DXRPT_KERNEL_LIB_DIR=ab/head6 run --label head6 --config $cfg
  done
  run --label now --share 8 --rank 2 --cur-copy
  DXRPT_KERNEL_LIB_DIR=ab/head6 run --label head6 --share 8 --rank 2 --cur-copy
done
