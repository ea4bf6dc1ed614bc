#!/bin/bash
# r03 final sequence: GPU suite + smoke + bench (gpu_check.sh), profiles of every config + bench lines
# (final_profiles.sh), every rank's share.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_check.sh > gpurun_out/gpu_check_final.txt 2>&1
rc=$?; tail -8 gpurun_out/gpu_check_final.txt | cut -c1-200
[ $rc -ne 0 ] && exit $rc
bash scripts/final_profiles.sh > gpurun_out/final_profiles.txt 2>&1 || { tail -5 gpurun_out/final_profiles.txt; exit 1; }
grep "per frame" gpurun_out/final_profiles.txt
bash scripts/shares_all_ranks.sh > gpurun_out/shares_all_ranks.txt 2>&1
