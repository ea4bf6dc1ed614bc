#!/bin/bash
# r03: cost-balanced bands (one census frame's per-band wave time, LPT) vs round-robin bands, every rank.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 240 python -u scripts/time_frames.py --rounds 3 --frames 32"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 0 1 2 3 4 5 6 7; do run --config metric --share 8 --rank $r --layout bands-balanced --label balanced; done
for r in 0 1 2 3; do run --config metric --share 4 --rank $r --layout bands-balanced --label balanced; done
for r in 0 1; do run --config metric --share 2 --rank $r --layout bands-balanced --label balanced; done
for r in 0 1 2 3 4 5 6 7; do run --config c5 --share 8 --rank $r --layout bands-balanced --label balanced; done
