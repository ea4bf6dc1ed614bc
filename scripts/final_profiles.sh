#!/bin/bash
# Final measurement (RND=<round>): rocprofv3 profiles of CONFIGS (kernel trace + PMC passes), then, with
# BENCH=1, the bench line of every config (scripts/bench_configs.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CONFIGS="${CONFIGS:-metric c2 c4 c3 c5}" STEPS=16 RND=${RND:-r06} bash scripts/profile_configs.sh > gpurun_out/profile_run_${RND:-r06}.log 2>&1 \
  || { echo "profiles failed"; tail -20 gpurun_out/profile_run_${RND:-r06}.log; exit 1; }
grep "per frame" gpurun_out/profile_run_${RND:-r06}.log
[ "${BENCH:-1}" = 1 ] && bash scripts/bench_configs.sh
exit 0
