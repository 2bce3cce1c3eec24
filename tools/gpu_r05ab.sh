#!/bin/bash
# Round-5 GPU step AB: cost of hs_cross's per-row tau at k = 64, by a build
# that computes it twice (exp/libocffm_tau2.so; the second product x 0).
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
for cfg in "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_tau2.so" "X=1" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_tau2.so" "X=1"; do
  env $cfg timeout -k 10 200 python tools/profile_epoch.py fp32 2 outbrain > $out/pe_ab.txt 2>&1
  echo "== $cfg"; grep -E "epoch wall|hs_cross|feat_hv" $out/pe_ab.txt | head -4
done
