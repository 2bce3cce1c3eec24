#!/bin/bash
# Round-5 GPU step AD: the gradient pass's grid at one resident wave of
# blocks (OCFFM_GD_FILL, default) against the fixed cap (OCFFM_GD_FILL=0) and
# other caps; the feature pass's cap; fp32 and fp64, kkbox shape.
set -e -o pipefail
bash tools/ab.sh 2 "X=1" "OCFFM_GD_FILL=0" "OCFFM_GD_FILL=0 OCFFM_GD_BLOCKS=1024" "OCFFM_GD_FILL=0 OCFFM_GD_BLOCKS=512" \
  "OCFFM_FEAT_BLOCKS=512"
cp gpurun_out/ab.txt gpurun_out/ab_ad32.txt
bash tools/ab64.sh 2 "X=1" "OCFFM_GD_FILL=0" "OCFFM_GD_FILL=0 OCFFM_GD_BLOCKS=1024" "OCFFM_GD_FILL=0 OCFFM_GD_BLOCKS=512" \
  "OCFFM_FEAT_BLOCKS=512"
