#!/bin/bash
# Round-5 GPU step X: bound probe of the fused id-field pass without its
# several-segment rows (exp/libocffm_xf1.so: they are skipped, timing only).
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
for cfg in "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_xf1.so" "OCFFM_XFUSE=0"; do
  env $cfg timeout -k 10 200 python tools/profile_epoch.py fp32 2 > $out/pe_x.txt 2>&1
  echo "== $cfg"; grep -E "epoch wall|hs_cross|feat_hv" $out/pe_x.txt | head -6
  env $cfg timeout -k 10 200 python tools/profile_epoch.py fp64 2 > $out/pe_x.txt 2>&1
  echo "== fp64 $cfg"; grep -E "epoch wall|hs_cross|feat_hv" $out/pe_x.txt | head -6
done
