#!/bin/bash
# r05: where the split schedule's time goes -- per-phase lane time of k_path_head and k_path_tail
# (ab/phases: -DDXRPT_DIAG_PHASES=1), metric, C3, C4 and a 1/8 share; then BVH build times on the host.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for cfg in metric c3 c4; do
  DXRPT_KERNEL_LIB_DIR=ab/phases timeout -k 10 120 python -u scripts/time_frames.py --label phases --config $cfg --rounds 3 --phases --opt FRAME_OVERLAP=0 || exit $?
done
DXRPT_KERNEL_LIB_DIR=ab/phases timeout -k 10 120 python -u scripts/time_frames.py --label phases --share 8 --rank 2 --rounds 3 --phases || exit $?
timeout -k 10 300 python -u scripts/bvh_build_times.py --threads 1,2,4,8,16,32 --repeat 2 || exit $?
