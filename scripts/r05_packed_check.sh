#!/bin/bash
# r05: packed normal / metallic / roughness taps (DXRPT_OPT_PACKED_TAPS) -- bit-identity tests, then
# every config with the option on (default) and off, same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "packed or retired or unknown or options" -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_packed.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_packed.log; [ $rc -ne 0 ] && exit $rc
run() { timeout -k 10 150 python -u scripts/time_frames.py --rounds 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1; }
for r in 1 2; do
  for cfg in metric c2 c4 c3; do
    run --label packed --config $cfg
    run --label packed-only --config $cfg --opt PACKED_TAPS=1
    run --label three-taps --config $cfg --opt PACKED_TAPS=0
  done
  for rk in 1 2; do
    run --label packed --share 8 --rank $rk --cur-copy
    run --label packed-only --share 8 --rank $rk --cur-copy --opt PACKED_TAPS=1
    run --label three-taps --share 8 --rank $rk --cur-copy --opt PACKED_TAPS=0
  done
done
