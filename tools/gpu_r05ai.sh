#!/bin/bash
# Round-5 GPU step AI: config-5 MFMA pass grids (rows_T blocks, Gram blocks),
# 2 M-row shard, per-family times.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
for cfg in "X=1" "OCFFM_TPRE_BLOCKS=512" "OCFFM_TPRE_BLOCKS=1024" "OCFFM_GRAM64_BLOCKS=2048" "OCFFM_GRAM64_BLOCKS=512"; do
  env $cfg timeout -k 10 300 python tools/profile_epoch.py fp32 1 cfg5 > $out/pe_ai.txt 2>&1
  echo "== $cfg"; grep -E "epoch wall|aggregates|rows_T|aggr_reduce" $out/pe_ai.txt | head -4
done
