#!/bin/bash
# Round-5 GPU step AP: positives per segment (OCFFM_SEG_LEN) and CG look-ahead
# after the resident-wave grids, fp32 and fp64 kkbox.
set -e -o pipefail
bash tools/ab.sh 2 "X=1" "OCFFM_SEG_LEN=24" "OCFFM_SEG_LEN=48" "OCFFM_SEG_LEN=64" "OCFFM_LOOKAHEAD=2"
cp gpurun_out/ab.txt gpurun_out/ab_ap32.txt
bash tools/ab64.sh 2 "X=1" "OCFFM_SEG_LEN=24" "OCFFM_SEG_LEN=48" "OCFFM_SEG_LEN=64"
