cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "traversal_variants or boxtest_256 or sponza_1080p_L3 or suntemple" > gpurun_out/pytest_variants.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_variants.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python scripts/ab_variants.py --frames 16 --rounds 3 --variants q0,q6,q7,q8,q6s128,q6s64 > gpurun_out/ab_shade.log 2>&1
