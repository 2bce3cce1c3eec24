#!/bin/bash
# Counter passes over one short bench run, restricted to the kernels named
# by the regex (default: the positive-gather and feature-pass kernels).
#   bash tools/pmc_passes.sh <tag> [regex]     (PMC_CMD overrides the program)
set -e -o pipefail
tag=${1:-x}
re=${2:-"k_hs_cross|k_feat|k_gd_cross|k_update_cross"}
out=gpurun_out/pmc_$tag
rm -rf $out && mkdir -p $out
export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
           "SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum" \
           "TA_BUSY_avr TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc --kernel-include-regex "$re" --output-format csv -d $out/p$i -o run \
    -- ${PMC_CMD:-python bench.py --steps 1 --warmup 1 --cpu-baseline off} > $out/p$i.log 2>&1
done
ls $out
