#!/bin/bash
# rocprofv3 PC sampling of the bench (hot instructions of k_path).  Outputs under gpurun_out/pcs/;
# summarise with scripts/pcsample_summary.py (maps PCs to the disassembly of libdxrpt.so's code object).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pcs
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/list_avail.txt 2>&1 || echo "list-avail rc=$?"
grep -i -A12 "pc sampl\|PC_SAMPL\|stochastic\|host_trap" $OUT/list_avail.txt | head -40
METHOD=${METHOD:-stochastic}
UNIT=${UNIT:-cycles}
INTERVAL=${INTERVAL:-1048576}
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $METHOD --pc-sampling-unit $UNIT \
    --pc-sampling-interval $INTERVAL -d $OUT/run -o pcs --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps ${STEPS:-16} --warmup 2 > $OUT/bench.json 2> $OUT/pcs.err
rc=$?
echo "pc sampling rc=$rc"
tail -5 $OUT/pcs.err
find $OUT/run -type f | head -20
exit $rc
