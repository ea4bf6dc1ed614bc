cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_steady_state.py tests/test_gpu_shipped.py tests/test_gpu_shipped_toggles.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_split15.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_split15.log; [ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 --cur-copy "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
run --label default --config c2
run --label nosplit --config c2 --opt MEGAKERNEL_SPLIT=0
run --label default --config c3 --share 8 --rank 2
run --label nosplit --config c3 --share 8 --rank 2 --opt MEGAKERNEL_SPLIT=0
done
