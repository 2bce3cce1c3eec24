#!/bin/bash
# Round-5 GPU step AG: resident-wave grids for the side gradient, update and
# column-Gram step passes (OCFFM_MISC_FILL): the suite, A/B fp32 / fp64
# kkbox, outbrain / kdd12 epochs.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/r05ag_pytest.log 2>&1 || { tail -40 $out/r05ag_pytest.log; exit 1; }
tail -1 $out/r05ag_pytest.log
bash tools/ab.sh 2 "X=1" "OCFFM_MISC_FILL=0"
bash tools/ab64.sh 2 "X=1" "OCFFM_MISC_FILL=0"
for shape in outbrain kdd12; do
  for cfg in "X=1" "OCFFM_MISC_FILL=0"; do
    env $cfg timeout -k 10 200 python tools/profile_epoch.py fp32 2 $shape > $out/pe_ag.txt 2>&1
    echo "== $shape $cfg"; grep -E "epoch wall|update|gd_side|hv_cgram" $out/pe_ag.txt | head -6
  done
done
