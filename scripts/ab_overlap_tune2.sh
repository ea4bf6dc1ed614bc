#!/bin/bash
# Second pass of the overlapped-frame retune: 64-lane waves and path order on the small shares.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 200 python -u scripts/time_frames.py --rounds 3 --frames 32"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for s in "--share 8 --rank 5" "--share 8 --rank 2" "--share 8 --rank 0"; do
  for occ in 4 5 6; do
    run --config metric $s --lanes 64 --occ $occ --wave-order 0 --label l64o0
    run --config metric $s --lanes 64 --occ $occ --label l64o2
  done
done
for occ in 5 6 7; do
  run --config metric --share 4 --rank 1 --occ $occ --wave-order 0 --label o0
  run --config metric --share 4 --rank 1 --occ $occ --label o2
done
for occ in 6 7; do
  run --config metric --share 2 --rank 1 --occ $occ --wave-order 0 --label o0
  run --config c2 --occ $occ --wave-order 0 --label o0
  run --config c5 --share 8 --rank 3 --occ $occ --wave-order 0 --label o0
done
run --config c5 --share 8 --rank 3 --occ 5 --wave-order 0 --label o0
run --config c3 --share 8 --rank 3 --label default
run --config c3 --share 8 --rank 3 --lanes 64 --wave-order 0 --label l64o0
run --config c3 --label default
run --config c5 --label default
