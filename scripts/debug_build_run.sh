#!/bin/bash
# The DXRPT_DEBUG kernel build (range checks on every queued path state a tail reads and every stage entry
# a blend reads) over every shipped overlapped schedule: tests/test_gpu_debug.py under ab/debug.
# Build first on the CPU host: make -C dxrpathtracer_amd/csrc variant NAME=debug EXTRA=-DDXRPT_DEBUG=1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
test -f ab/debug/libdxrpt.so || { echo "ab/debug/libdxrpt.so missing"; exit 2; }
DXRPT_KERNEL_LIB_DIR=ab/debug timeout -k 10 600 python -u -m pytest tests/test_gpu_debug.py tests/test_gpu_steady_state.py::test_overlapped_order_rebuilds_are_bit_identical \
  -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/debug_build.log 2>&1
rc=$?; echo "debug-build pytest rc=$rc"; grep -E "debug build:|passed|failed|Error" gpurun_out/debug_build.log | tail -20
exit $rc
