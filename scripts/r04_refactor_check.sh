#!/bin/bash
# r04: the ABI-3 refactor on the GPU -- suite, smoke, bench, then the refactored build against the r03 build
# (ab/head) on the metric, C2, C3 and a 1/8 share, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r04a bash scripts/gpu_check.sh || exit $?
for cfg in "--config metric" "--config c2" "--config c3 --frames 16" "--config metric --share 8 --rank 5" "--config c4"; do
  BUILDS="ab/head dxrpathtracer_amd/lib" ROUNDS=2 bash scripts/ab_builds.sh $cfg --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
done
