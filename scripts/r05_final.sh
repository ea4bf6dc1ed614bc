#!/bin/bash
# r05 final: GPU tests, rocprofv3 profiles of every config (kernel trace + PMC passes, summarised into
# profiles/r05_*), every config through bench.py, every rank's share.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/pytest_final.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|overall max" gpurun_out/pytest_final.log | tail -3; [ $rc -ne 0 ] && exit $rc
CONFIGS="metric c2 c4 c3 c5" STEPS=16 RND=r05 bash scripts/profile_configs.sh > gpurun_out/profile_all_final.log 2>&1 \
  || { echo "profiles failed"; tail -20 gpurun_out/profile_all_final.log; exit 1; }
grep -E "k_path" gpurun_out/profile_all_final.log | cut -c1-200
bash scripts/bench_configs.sh || exit 1
SHARE_FLAGS=--cur-copy bash scripts/shares_all_ranks.sh > gpurun_out/r05_shares_all_ranks_final.txt 2>&1 || exit 1
echo done
