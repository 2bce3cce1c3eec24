#!/bin/bash
# Round-5 GPU step M: the suite with the reduce-scatter dot products, then
# A/B against the round-4 subgroup sums (exp/libocffm_rs0.so), fp32 and fp64.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/r05m_pytest.log 2>&1 || { tail -40 $out/r05m_pytest.log; exit 1; }
tail -2 $out/r05m_pytest.log
bash tools/ab.sh 3 "X=1" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_rs0.so"
bash tools/ab64.sh 2 "X=1" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_rs0.so"
for cfg in "X=1" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_rs0.so"; do
  env $cfg timeout -k 10 200 python tools/profile_epoch.py fp32 2 > $out/pe_m.txt 2>&1
  echo "== $cfg"; grep -E "epoch wall|hs_cross_row|gd_cross_row|feat_hv|hs_side" $out/pe_m.txt | head -8
  env $cfg timeout -k 10 200 python tools/profile_epoch.py fp32 2 outbrain > $out/pe_m.txt 2>&1
  echo "== outbrain $cfg"; grep -E "epoch wall|hs_cross_row|gd_cross_row|feat_hv|hs_side" $out/pe_m.txt | head -8
done
