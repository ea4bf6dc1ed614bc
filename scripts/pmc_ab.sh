#!/bin/bash
# PMC A/B of kernel builds: one rocprofv3 --pmc pass per (build, counter group) over a short
# time_frames.py run; writes gpurun_out/pmcab/<build>_<group>/ and prints per-kernel averages.
# usage: BUILDS="ab/x dxrpathtracer_amd/lib" bash scripts/pmc_ab.sh [time_frames args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcab
mkdir -p $OUT
GROUPS_=${PMC_GROUPS:-"SQC_ICACHE_HITS,SQC_ICACHE_MISSES,SQ_IFETCH,SQ_IFETCH_LEVEL,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_INSTS_VALU,SQ_BUSY_CYCLES"}
for b in ${BUILDS:-dxrpathtracer_amd/lib}; do
  for g in $GROUPS_; do
    tag=$(echo "$b" | tr '/' '_')_$(echo $g | cut -c1-24)
    DXRPT_KERNEL_LIB_DIR=$b timeout -s KILL 90 rocprofv3 --pmc $(echo $g | tr ',' ' ') -d $OUT/$tag -o run \
        --output-format csv -- python3 scripts/time_frames.py --rounds 1 --frames 8 --label "$b" "$@" \
        > $OUT/$tag.log 2>&1 || { echo "pmc $b $g failed rc=$?"; tail -3 $OUT/$tag.log; exit 1; }
    python3 scripts/pmc_ab_summary.py $OUT/$tag "$b" || exit 1
  done
done
