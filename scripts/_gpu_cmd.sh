cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "traversal_variants or boxtest_256 or sponza_1080p_L3 or suntemple" > gpurun_out/pytest_variants.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_variants.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python scripts/ab_variants.py --frames 16 --rounds 3 --variants n0,n73,n128,n256,n0b256,n73b256,n256b256,n512b256,n128b128 > gpurun_out/ab_lds.log 2>&1
