#!/bin/bash
# r04: bench (schedule-pinned frame-at-a-time pass) then the in-tree build against ab/* builds,
# interleaved, on the configs in $AB_CONFIGS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 32 > gpurun_out/bench_${TAG:-r04}.json 2> gpurun_out/bench_${TAG:-r04}.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench_${TAG:-r04}.err; exit 1; }
cat gpurun_out/bench_${TAG:-r04}.json
IFS=';' read -ra CFGS <<< "${AB_CONFIGS:-"--config metric;--config c3 --frames 16;--config metric --share 8 --rank 5"}"
for cfg in "${CFGS[@]}"; do
  BUILDS=${BUILDS:-"ab/head dxrpathtracer_amd/lib"} ROUNDS=2 bash scripts/ab_builds.sh $cfg --rounds 3 --kernels 2>&1 | grep -v amdgpu.ids || exit 1
done
