#!/bin/bash
# Schedule knobs re-tuned under overlapped frames (DXRPT_OPT_FRAME_OVERLAP 1, the default): lanes per
# wave, cost order, occupancy on the band shares and the full frames.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 200 python -u scripts/time_frames.py --rounds 3 --frames 32"
run() { $T "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for s in "--share 8 --rank 5" "--share 8 --rank 2"; do
  run --config metric $s --label default
  run --config metric $s --lanes 64 --label lanes64
  run --config metric $s --lanes 64 --occ 7 --label lanes64
  run --config metric $s --wave-order 0 --label order0
  run --config metric $s --occ 6 --label occ6
  run --config metric $s --occ 4 --label occ4
done
for s in "--share 4 --rank 1" "--share 2 --rank 1"; do
  run --config metric $s --label default
  run --config metric $s --wave-order 0 --label order0
  run --config metric $s --occ 7 --label occ7
  run --config metric $s --occ 6 --label occ6
done
for c in metric c4 c2; do
  run --config $c --label default
  run --config $c --wave-order 1 --label order1
  run --config $c --wave-order 0 --label order0
  run --config $c --occ 6 --label occ6
  run --config $c --occ 8 --label occ8
done
run --config c5 --share 8 --rank 3 --label default
run --config c5 --share 8 --rank 3 --wave-order 0 --label order0
run --config c5 --share 8 --rank 3 --occ 6 --label occ6
