#!/bin/bash
# r05 final (after the 256-frame order period): GPU tests, every rank's share, the metric bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/pytest_final3.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|overall max" gpurun_out/pytest_final3.log | tail -3; [ $rc -ne 0 ] && exit $rc
SHARE_FLAGS=--cur-copy bash scripts/shares_all_ranks.sh > gpurun_out/r05_shares_all_ranks_final.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 32 --warmup 5 > gpurun_out/bench_final3.json 2> gpurun_out/bench_final3.err || exit 1
cat gpurun_out/bench_final3.json | cut -c1-300
