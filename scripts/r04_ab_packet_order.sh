#!/bin/bash
# r04 A/B: the packet (wave-coherent) any-hit traversal -- the head's depth-1 sun shadow rays -- back near to far
# while per-lane any-hit rays stay far to near (ab/pn, built with the since-removed -DDXRPT_PACKET_ANYHIT_FAR=0)
# against the in-tree build of the time (far to near for both).  Recorded run: profiles/r04_ab_packet_order.txt;
# the order is now traverse8_packet's kFar template argument (near to far in k_path at <= 5 waves/SIMD).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
DXRPT_KERNEL_LIB_DIR=ab/pn timeout -k 10 700 python -u -m pytest tests/test_gpu_shipped.py tests/test_gpu_edge_sizes.py \
    -q -x --timeout 300 --timeout-method thread > gpurun_out/pn_parity.log 2>&1
rc=$?; echo "pn parity rc=$rc"; tail -2 gpurun_out/pn_parity.log; [ $rc -ne 0 ] && exit $rc
T="timeout -k 10 150 python -u scripts/time_frames.py --rounds 3"
for cfg in "--config metric" "--config c2" "--config c3 --frames 16" "--config c4" "--config c5 --frames 8" "--config metric --share 8 --rank 2" "--config metric --share 8 --rank 7"; do
  for r in 1 2; do
    for b in dxrpathtracer_amd/lib ab/pn; do
      DXRPT_KERNEL_LIB_DIR=$b $T $cfg --label $b 2>> gpurun_out/ab_packet_order.err
      rc=$?; [ $rc -ne 0 ] && { echo "$b $cfg rc=$rc"; [ $rc -gt 1 ] && exit $rc; }
    done
  done
done
exit 0
