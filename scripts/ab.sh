#!/bin/bash
# Interleaved A/B of kernel builds and options on one GPU box (the one A/B driver; r01-r05's one-off
# r0*_ab_*.sh scripts are folded into it, their records indexed in profiles/AB_INDEX.md).
#   BUILDS  build directories holding a libdxrpt.so (default: every ab/*/ plus the in-tree lib)
#   CASES   ';'-separated scripts/time_frames.py argument sets (default: the metric, C4, C3, C2 and a 1/8 share)
#   ROUNDS  interleaving rounds (default 2)
# Extra arguments go to every time_frames.py call.  Each call runs in its own process under a time limit;
# the first failure ends the run (no retries).  Example:
#   BUILDS="ab/base dxrpathtracer_amd/lib" CASES="--config metric;--share 8 --rank 2" scripts/ab.sh --rounds 5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BUILDS=${BUILDS:-"$(ls -d ab/*/ 2>/dev/null | tr '\n' ' ') dxrpathtracer_amd/lib"}
CASES=${CASES:-"--config metric;--config c4;--config c3;--config c2;--share 8 --rank 2"}
IFS=';' read -r -a CASE_LIST <<< "$CASES"
for r in $(seq 1 "${ROUNDS:-2}"); do
  for c in "${CASE_LIST[@]}"; do
    for b in $BUILDS; do
      # shellcheck disable=SC2086
      DXRPT_KERNEL_LIB_DIR=$b timeout -k 10 180 python -u scripts/time_frames.py --label "$b" $c "$@" || exit $?
    done
  done
done
