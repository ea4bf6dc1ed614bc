cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_exp3.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|overall max" gpurun_out/pytest_exp3.log | tail -3
[ $rc -ne 0 ] && exit $rc
ROUNDS=2 bash scripts/ab.sh > gpurun_out/ab_exp3.txt 2>&1; echo "ab rc=$?"
