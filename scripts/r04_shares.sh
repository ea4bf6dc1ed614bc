#!/bin/bash
# r04: every rank's 1/8 band share of the metric frame (the 8-GPU tail) with the shipped defaults and a
# few schedule alternatives, then the 1/4 and 1/2 shares: one MI355X, no gather.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 120 python -u scripts/time_frames.py --rounds 3 --frames 32"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
run --config metric --label default
for r in 0 1 2 3 4 5 6 7; do run --config metric --share 8 --rank $r --label default; done
# DEFAULT_ONLY=1: the shipped defaults only (every rank of the 1/8, 1/4 and 1/2 shares)
[ -z "$DEFAULT_ONLY" ] && for alt in "WAVE_ORDER=0" "MEGAKERNEL_OCCUPANCY=5" "MEGAKERNEL_OCCUPANCY=6" "MEGAKERNEL_SPLIT=1"; do
  for r in 0 1 2 3 4 5 6 7; do run --config metric --share 8 --rank $r --label "$alt" --opt $alt; done
done
[ -z "$DEFAULT_ONLY" ] && for r in 0 1 2 3 4 5 6 7; do run --config metric --share 8 --rank $r --layout blocks --label blocks; done
for r in 0 1 2 3; do run --config metric --share 4 --rank $r --label default; done
for r in 0 1; do run --config metric --share 2 --rank $r --label default; done
