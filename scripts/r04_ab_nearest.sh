#!/bin/bash
# r04 A/B: per-lane closest-hit traversal descends into the nearest internal child first (exact entry distance),
# the node's other hit children stay one octant-ordered group (ab/nf, built with the since-removed
# -DDXRPT_NEAREST_FIRST=1: every per-lane closest hit) against the in-tree build of the time.  Recorded run:
# profiles/r04_ab_nearest.txt; the order is now the kNearest template argument of traverse8.  Parity of the
# variant first, then two interleaved timing passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
DXRPT_KERNEL_LIB_DIR=ab/nf timeout -k 10 700 python -u -m pytest tests/test_gpu_shipped.py tests/test_gpu_edge_sizes.py \
    tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread > gpurun_out/nf_parity.log 2>&1
rc=$?; echo "nf parity rc=$rc"; tail -2 gpurun_out/nf_parity.log; [ $rc -ne 0 ] && exit $rc
T="timeout -k 10 150 python -u scripts/time_frames.py --rounds 3"
for cfg in "--config metric" "--config c2" "--config c3 --frames 16" "--config c4" "--config c5 --frames 8" "--config metric --share 8 --rank 2" "--config metric --share 8 --rank 7"; do
  for r in 1 2; do
    for b in dxrpathtracer_amd/lib ab/nf; do
      DXRPT_KERNEL_LIB_DIR=$b $T $cfg --label $b 2>> gpurun_out/ab_nearest.err
      rc=$?; [ $rc -ne 0 ] && { echo "$b $cfg rc=$rc"; [ $rc -gt 1 ] && exit $rc; }
    done
  done
done
exit 0
