#!/bin/bash
# Round-5 GPU step AS: fp64 hs_cross at 4 waves per SIMD (exp hso4: 128
# registers with spills; hsg4: 4 gathers per round, 128 registers).
set -e -o pipefail
bash tools/ab64.sh 2 "X=1" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_hso4.so" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_hsg4.so"
