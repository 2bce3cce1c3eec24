#!/bin/bash
# Round-5 GPU step L: the suite; outbrain with the short pass and the T pre-pass.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/r05l_pytest.log 2>&1 || { tail -40 $out/r05l_pytest.log; exit 1; }
tail -2 $out/r05l_pytest.log
for cfg in "OCFFM_SHORTPASS=0" "OCFFM_X=1" "OCFFM_TPRE=1"; do
  env $cfg timeout -k 10 200 python tools/profile_epoch.py fp32 2 outbrain > $out/pe_ob_l.txt 2>&1
  echo "== $cfg"; grep -E "epoch wall|hs_cross_row|gd_cross_row|rows_T|feat_hv|hs_side" $out/pe_ob_l.txt | head -8
done
