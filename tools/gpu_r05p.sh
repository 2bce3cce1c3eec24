#!/bin/bash
# Round-5 GPU step P: the CG direction formed once per step (k_cg_dir) for
# row passes with > 2 node references per column: the suite, then
# OCFFM_DIRPRE=0 / default per shape.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/r05p_pytest.log 2>&1 || { tail -40 $out/r05p_pytest.log; exit 1; }
tail -1 $out/r05p_pytest.log
bash tools/ab.sh 2 "X=1" "OCFFM_DIRPRE=0"
for shape in kkbox kdd12 outbrain; do
  for cfg in "X=1" "OCFFM_DIRPRE=0"; do
    env $cfg timeout -k 10 200 python tools/profile_epoch.py fp32 2 $shape > $out/pe_p_${shape}_${cfg%%=*}.txt 2>&1
    echo "== $shape $cfg"; grep -E "epoch wall|hs_cross_row|cg_dir|feat_hv|hs_side" $out/pe_p_${shape}_${cfg%%=*}.txt | head -6
  done
done
