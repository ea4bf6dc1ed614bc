#!/bin/bash
# r04 A/B: packet (wave-coherent) closest-hit traversal -- the primary rays -- descends first into the nearest hit
# internal child of the block's middle lane, the rest of the union as one octant group (ab/pk: make -C
# dxrpathtracer_amd/csrc variant NAME=pk EXTRA=-DDXRPT_PACKET_NEAREST=1) against octant order (in-tree build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
DXRPT_KERNEL_LIB_DIR=ab/pk timeout -k 10 700 python -u -m pytest tests/test_gpu_shipped.py tests/test_gpu_edge_sizes.py \
    -q -x --timeout 300 --timeout-method thread > gpurun_out/pk_parity.log 2>&1
rc=$?; echo "pk parity rc=$rc"; tail -2 gpurun_out/pk_parity.log; [ $rc -ne 0 ] && exit $rc
T="timeout -k 10 150 python -u scripts/time_frames.py --rounds 3"
for cfg in "--config metric" "--config c2" "--config c3 --frames 16" "--config c4" "--config c5 --frames 8" "--config metric --share 8 --rank 2" "--config metric --share 8 --rank 7"; do
  for r in 1 2; do
    for b in dxrpathtracer_amd/lib ab/pk; do
      DXRPT_KERNEL_LIB_DIR=$b $T $cfg --label $b 2>> gpurun_out/ab_packet_nearest.err
      rc=$?; [ $rc -ne 0 ] && { echo "$b $cfg rc=$rc"; [ $rc -gt 1 ] && exit $rc; }
    done
  done
done
exit 0
