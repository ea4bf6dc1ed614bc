#!/bin/bash
# r03 final: shipped/steady-state parity of the build, then every BASELINE config through bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_shipped.py tests/test_gpu_steady_state.py -m gpu -q -x -rf \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_final_cfg.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_final_cfg.log | tail -5
[ $rc -ne 0 ] && exit $rc
bash scripts/bench_configs.sh
