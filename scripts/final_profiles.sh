#!/bin/bash
# r03 final: rocprofv3 profiles of every config (kernel trace + PMC passes), then the bench line of every config.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CONFIGS="metric c2 c4 c3 c5" STEPS=16 RND=r03 bash scripts/profile_configs.sh > gpurun_out/profile_all_run.log 2>&1 \
  || { echo "profiles failed"; tail -20 gpurun_out/profile_all_run.log; exit 1; }
grep "per frame" gpurun_out/profile_all_run.log
bash scripts/bench_configs.sh
