#!/bin/bash
# Round-5 GPU step Q: bound probe of hs_cross's per-segment tau term
# (exp/libocffm_notau.so skips it: timing only, wrong numerics).
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
for shape in outbrain kdd12; do
  for cfg in "X=1" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_notau.so"; do
    env $cfg timeout -k 10 200 python tools/profile_epoch.py fp32 2 $shape > $out/pe_q.txt 2>&1
    echo "== $shape $cfg"; grep -E "epoch wall|hs_cross_row|feat_hv|hs_side" $out/pe_q.txt | head -5
  done
done
