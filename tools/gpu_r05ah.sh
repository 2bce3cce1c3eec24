#!/bin/bash
# Round-5 GPU step AH: fp64 side-row grid at its resident wave, and the fp64
# gradient pass's occupancy bound (exp builds: gd occupancy 2 / 4).
set -e -o pipefail
bash tools/ab64.sh 2 "X=1" "OCFFM_SIDE_FILL=1" "OCFFM_ROW_FILL=1 OCFFM_SIDE_FILL=1"
