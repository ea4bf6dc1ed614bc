#!/bin/bash
# Concurrent frame parts (scripts/ab_split.py) with the single and the depth-split megakernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T="timeout -k 10 300 python -u scripts/ab_split.py --rounds 2 --frames 16 --parts ${PARTS:-1,2}"
for c in ${CONFIGS:-c3 c5 metric}; do
  for pl in ${LAYOUTS:-bands halves}; do
    $T --config $c --part-layout $pl --msplit 1 --occ 6 --tail-occ 7 --wave-order 0 || exit 1
  done
done
