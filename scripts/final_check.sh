#!/bin/bash
# r03 final: GPU suite + smoke + bench (scripts/gpu_check.sh), then every rank's share.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_check.sh > gpurun_out/gpu_check.txt 2>&1
rc=$?; cat gpurun_out/gpu_check.txt | tail -12
[ $rc -ne 0 ] && exit $rc
bash scripts/shares_all_ranks.sh > gpurun_out/shares_all_ranks.txt 2>&1
