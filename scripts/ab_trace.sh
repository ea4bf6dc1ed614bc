#!/bin/bash
# Per-dispatch kernel durations (rocprofv3 kernel trace) of the in-process A/B driver, one variant
# per process so dispatches group cleanly; summarise with scripts/ab_trace_summary.py.
#   VARIANTS="w8m0 w8m1r16k4p16" bash scripts/ab_trace.sh [tag]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-abtrace}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for v in ${VARIANTS}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/$v -o run --output-format csv -- \
      python3 scripts/ab_variants.py --variants $v --rounds 1 --frames 8 > $OUT/$v.log 2>&1
  rc=$?
  echo "variant $v rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $OUT/$v.log; exit $rc; }
done
exit 0
