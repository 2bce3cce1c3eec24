#!/bin/bash
# Round-5 GPU step U: the in-block gradient pass reading the stored values
# through perm (default) against a refresh pass of the item orientation
# (OCFFM_YTVIA=0), kkbox shape.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
bash tools/ab.sh 3 "X=1" "OCFFM_YTVIA=0"
for cfg in "X=1" "OCFFM_YTVIA=0"; do
  env $cfg timeout -k 10 200 python tools/profile_epoch.py fp32 2 > $out/pe_u.txt 2>&1
  echo "== $cfg"; grep -E "epoch wall|gd_cross_row|refresh_base|flush" $out/pe_u.txt | head -5
done
