#!/bin/bash
# Round-5 GPU step T: vector-memory pipeline counters (TA / TCP / TCC) of the
# positive-gather passes at kkbox shape, one pass per counter pair.
set -e -o pipefail
out=gpurun_out/pmct_r05t
rm -rf $out && mkdir -p $out
export TMPDIR=/tmp
re="k_gd_cross_seg|k_hs_cross_seg"
i=0
for pmc in "GRBM_GUI_ACTIVE TA_BUSY_avr" "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum" \
           "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum" "TCC_HIT_sum TCC_MISS_sum" \
           "TA_BUFFER_READ_WAVEFRONTS_sum TA_TA_BUSY_sum" "TCC_EA0_RDREQ_sum TCC_TAG_STALL_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "$re" --output-format csv -d $out/p$i -o run \
    -- python bench.py --steps 1 --warmup 1 --cpu-baseline off --modes off --sgd off > $out/p$i.log 2>&1
done
python tools/pmc_kernels.py $(find $out -name '*counter_collection.csv') > gpurun_out/r05t_tcp.txt
wc -l gpurun_out/r05t_tcp.txt
