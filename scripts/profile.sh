#!/bin/bash
# rocprofv3 passes over the bench (kernel trace + stats, then one PMC group per pass; never combined
# with other tracing domains).  CONFIG=metric|c2|c3|c4|c5 (bench.py --config).  Outputs under
# gpurun_out/prof_<config>/; summarise with
#   PMC_CONFIG_TAG=<config> PMC_CONFIG="<scene>-proxy WxH L=n" scripts/pmc_summary.py gpurun_out/prof_<config> <round>
# (bench.py's frame-at-a-time pass runs on the caller's stream: pmc_summary.py reads those launches as the
# per-launch durations / counters of the bench line's roofline.)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${CONFIG:-metric}
OUT=gpurun_out/prof_$CFG
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --config $CFG"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- $B --steps ${STEPS:-32} --warmup 5 \
    > $OUT/kt_bench.json 2> $OUT/kt.err || exit $?
echo "kernel trace ok"; cat $OUT/kt_bench.json
for pmc in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM" "SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_WAIT_INST_LDS"; do
  tag=$(echo $pmc | tr ' ' '_')
  timeout -s KILL 300 rocprofv3 --pmc $pmc -d $OUT/pmc_$tag -o run --output-format csv -- $B --steps 8 --warmup 2 \
      > $OUT/pmc_$tag.json 2> $OUT/pmc_$tag.err || { echo "pmc $pmc failed rc=$?"; tail -5 $OUT/pmc_$tag.err; exit 1; }
  echo "pmc $pmc ok"
done
