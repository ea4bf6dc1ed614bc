#!/bin/bash
# r05 A/B, same box, interleaved: ab/nochain (r05 builder, slot-by-slot shadow loop, taps one by one),
# ab/nobatch (+ the last depth's two shadow rays chained in one traversal loop), in-tree (+ a hit's five
# material taps issuing their 20 texel loads together).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 120 python -u scripts/time_frames.py --rounds 5 "$@" || exit $?; }
for r in 1 2; do
  for cfg in metric c4 c3 c2; do
    for b in ab/nochain ab/nobatch dxrpathtracer_amd/lib; do DXRPT_KERNEL_LIB_DIR=$b run --label $b --config $cfg; done
  done
  for b in ab/nochain ab/nobatch dxrpathtracer_amd/lib; do DXRPT_KERNEL_LIB_DIR=$b run --label $b --share 8 --rank 2; done
done
