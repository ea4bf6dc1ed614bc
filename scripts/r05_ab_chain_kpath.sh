#!/bin/bash
# r05 A/B, same box, interleaved: chained shadow rays in k_path at <= 5 waves/SIMD (the band shares) and in
# the last-depth tails (in-tree) against ab/nochain (-DDXRPT_CHAIN_SHADOWS=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { timeout -k 10 120 python -u scripts/time_frames.py --rounds 5 "$@" || exit $?; }
for r in 1 2; do
  for rk in 2 5 7; do for b in ab/nochain dxrpathtracer_amd/lib; do DXRPT_KERNEL_LIB_DIR=$b run --label $b --share 8 --rank $rk; done; done
  for rk in 1 3; do for b in ab/nochain dxrpathtracer_amd/lib; do DXRPT_KERNEL_LIB_DIR=$b run --label $b --share 4 --rank $rk; done; done
  for b in ab/nochain dxrpathtracer_amd/lib; do DXRPT_KERNEL_LIB_DIR=$b run --label $b --share 2 --rank 1; done
  for b in ab/nochain dxrpathtracer_amd/lib; do DXRPT_KERNEL_LIB_DIR=$b run --label $b --config metric; done
  for b in ab/nochain dxrpathtracer_amd/lib; do DXRPT_KERNEL_LIB_DIR=$b run --label $b --config c5 --share 8 --rank 3; done
done
