#!/bin/bash
# Packet traversal modes (DXRPT_OPT_PACKET_TRAVERSAL: bit 0 primaries, bit 1 depth-1 sun shadows) on the
# band shares that set the N-GPU span, plus the full frame.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 200 python -u scripts/time_frames.py --rounds 3 --frames 24"
for pk in 3 2 1 0; do
  for args in "--config metric --share 8 --rank 5" "--config metric --share 8 --rank 2" "--config metric --share 4 --rank 1" "--config metric"; do
    $T $args --packet $pk --label packet$pk 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
