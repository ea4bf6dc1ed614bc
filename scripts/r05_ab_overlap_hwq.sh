#!/bin/bash
# r05: frames in flight with GPU_MAX_HW_QUEUES=8 (the runtime default is 4 hardware queues per process:
# a caller stream, 3-4 overlap slot streams and a gather side stream share them), with the side stream.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
export GPU_MAX_HW_QUEUES=8
for r in 1 2; do
  for o in 1 2 3; do
    run --label hwq8-ovl$o --share 8 --rank 2 --opt FRAME_OVERLAP=$o --side-stream
    run --label hwq8-ovl$o --share 8 --rank 7 --opt FRAME_OVERLAP=$o --side-stream
    run --label hwq8-ovl$o --share 4 --rank 2 --opt FRAME_OVERLAP=$o --side-stream
    run --label hwq8-ovl$o --share 2 --rank 0 --opt FRAME_OVERLAP=$o --side-stream
    run --label hwq8-ovl$o --config metric --opt FRAME_OVERLAP=$o
    run --label hwq8-ovl$o --config c2 --opt FRAME_OVERLAP=$o
  done
done
