#!/bin/bash
# GPU-box check: parity tests, smoke, a short bench.  Stops at the first crash/timeout (rc > 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-32}
TAG=${TAG:-check}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|overall max|FAILED|Error" gpurun_out/pytest_$TAG.log | tail -15
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps $STEPS --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
exit $rc
