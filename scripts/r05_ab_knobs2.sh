#!/bin/bash
# r05 late: runtime knobs re-swept on the final kernels -- XCD chunk (default 8) and packet traversal
# (default 3: packet primaries + packet depth-1 sun shadows).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for cfg in metric c4; do
    run --label default --config $cfg
    for x in 0 4 16; do run --label xcd$x --config $cfg --opt XCD_CHUNK=$x; done
    for p in 1 2; do run --label packet$p --config $cfg --opt PACKET_TRAVERSAL=$p; done
  done
  run --label default --share 8 --rank 2 --cur-copy
  for x in 0 4 16; do run --label xcd$x --share 8 --rank 2 --cur-copy --opt XCD_CHUNK=$x; done
done
