cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
DXRPT_KERNEL_LIB_DIR=ab/sexp timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_exp10.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|overall max" gpurun_out/pytest_exp10.log | tail -3
[ $rc -ne 0 ] && exit $rc
BUILDS="ab/sexp dxrpathtracer_amd/lib" ROUNDS=3 bash scripts/ab.sh > gpurun_out/ab_exp10.txt 2>&1; echo "ab rc=$?"
