#!/bin/bash
# The round's final measurement on one GPU box, in two calls (each well inside gpurun's 20-minute limit):
#   STAGE=1: GPU tests + smoke + the driver's bench command (scripts/gpu_check.sh), every config's bench line
#            (scripts/bench_configs.sh), every rank's share (scripts/shares_all_ranks.sh)
#   STAGE=2: rocprofv3 kernel trace + PMC passes of every config (scripts/final_profiles.sh, RND=r06), the
#            DXRPT_DEBUG build's range checks (scripts/debug_build_run.sh; build ab/debug first)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${STAGE:-1}" = 1 ]; then
  TAG=${TAG:-final} STEPS=20 bash scripts/gpu_check.sh || exit $?
  bash scripts/bench_configs.sh || exit 1
  bash scripts/shares_all_ranks.sh > gpurun_out/shares_all_ranks_final.txt 2>&1; echo "shares rc=$?"
else
  CONFIGS="metric c2 c4 c3 c5" BENCH=0 RND=${RND:-r06} bash scripts/final_profiles.sh || exit 1
  bash scripts/debug_build_run.sh
fi
