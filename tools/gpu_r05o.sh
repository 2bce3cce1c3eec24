#!/bin/bash
# Round-5 GPU step O: non-temporal position streams (exp/libocffm_nt.so;
# ntst: + non-temporal h stores) against the default build.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
bash tools/ab.sh 2 "X=1" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_nt.so" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_ntst.so"
for shape in kkbox kdd12 outbrain; do
  for cfg in "X=1" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_nt.so"; do
    env $cfg timeout -k 10 200 python tools/profile_epoch.py fp32 2 $shape > $out/pe_o.txt 2>&1
    echo "== $shape $cfg"; grep -E "epoch wall|hs_cross_row|gd_cross_row|feat_hv|hs_side" $out/pe_o.txt | head -6
  done
done
