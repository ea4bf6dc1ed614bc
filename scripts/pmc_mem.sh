#!/bin/bash
# Memory-pipeline counters (TA/TD/TCP, VMEM latency) over the bench, one rocprofv3 --pmc pass each.
# Outputs under gpurun_out/pmc_mem/; summarise with scripts/pmc_mem_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_mem
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --steps 8 --warmup 2"
i=0
PASSES=${PASSES:-default}
if [ "$PASSES" = "sq" ]; then
  set -- "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
         "SQ_WAVES SQ_INSTS_SMEM_NORM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE"
else
  set -- "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum" \
           "TD_TD_BUSY_sum TD_TC_STALL_sum" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum" \
           "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_REQUEST_sum" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INST_CYCLES_VMEM_RD" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"
fi
for pmc in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d $OUT/p$i -o run --output-format csv -- $B > $OUT/p$i.json 2> $OUT/p$i.err \
      || { echo "pmc pass $i ($pmc) failed rc=$?"; tail -5 $OUT/p$i.err; exit 1; }
  echo "pass $i ok: $pmc"
done
