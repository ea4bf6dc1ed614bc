#!/bin/bash
# One rocprofv3 --pmc pass per counter group (never combined with other tracing domains) over
# the in-process A/B driver on the bench workload.  Stops at the first crash / timeout.
#   PMC_GROUPS="G1;G2;..." bash scripts/pmc_sweep.sh [tag]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-sweep}
OUT=gpurun_out/$TAG
mkdir -p $OUT
VARIANT=${VARIANT:-w8m0}
rocprofv3 -L > $OUT/counters_avail.txt 2>&1 || true
IFS=';' read -ra GROUPS_ <<< "${PMC_GROUPS}"
i=0
for g in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $g -d $OUT/p$i -o run --output-format csv -- \
      python3 scripts/ab_variants.py --variants $VARIANT --rounds 1 --frames 8 > $OUT/p$i.log 2>&1
  rc=$?
  echo "group $i [$g] rc=$rc"
  case $rc in 124|134|137|139) tail -5 $OUT/p$i.log; exit $rc;; esac
  [ $rc -ne 0 ] && tail -3 $OUT/p$i.log
done
exit 0
