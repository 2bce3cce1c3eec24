#!/bin/bash
# Round-5 GPU step AF: resident-wave grids for the Hessian-vector row passes
# (OCFFM_ROW_FILL): A/B fp32 / fp64 kkbox, then outbrain and kdd12 epochs.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
bash tools/ab.sh 2 "X=1" "OCFFM_ROW_FILL=0"
bash tools/ab64.sh 2 "X=1" "OCFFM_ROW_FILL=0"
for shape in outbrain kdd12; do
  for cfg in "X=1" "OCFFM_ROW_FILL=0"; do
    env $cfg timeout -k 10 200 python tools/profile_epoch.py fp32 2 $shape > $out/pe_af.txt 2>&1
    echo "== $shape $cfg"; grep -E "epoch wall|hs_cross|hs_side|feat_hv" $out/pe_af.txt | head -5
  done
done
