#!/bin/bash
# Round-5 GPU step AC: fp64 grid caps (gd / hs / feature passes) at kkbox shape.
set -e -o pipefail
bash tools/ab64.sh 2 "X=1" "OCFFM_GD_BLOCKS=1024" "OCFFM_GD_BLOCKS=4096" "OCFFM_HS_BLOCKS=2048" "OCFFM_HS_BLOCKS=8192" \
  "OCFFM_FEAT_BLOCKS=2048" "OCFFM_FEAT_BLOCKS=512"
