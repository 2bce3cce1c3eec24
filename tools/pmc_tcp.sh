#!/bin/bash
# Vector-memory pipeline counters (TA / TCP / UTCL1) for one kernel family.
#   bash tools/pmc_tcp.sh <tag> <kernel regex>
set -e -o pipefail
tag=${1:-x}
re=${2:-"k_hs_cross"}
out=gpurun_out/pmct_$tag
rm -rf $out && mkdir -p $out
export TMPDIR=/tmp
i=0
for pmc in "GRBM_GUI_ACTIVE TA_BUSY_avr" "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum" \
           "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $pmc --kernel-include-regex "$re" --output-format csv -d $out/p$i -o run \
    -- python bench.py --steps 1 --warmup 1 --cpu-baseline off > $out/p$i.log 2>&1
done
