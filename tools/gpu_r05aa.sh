#!/bin/bash
# Round-5 GPU step AA: per-epoch wall times over 25 epochs (kdd12 / kkbox /
# outbrain), and a bound probe of hs_cross's per-row tau at k = 64
# (exp/libocffm_tauq.so: the QTQ product replaced by a diagonal stand-in,
# timing only).
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/epoch_times.py kdd12 25 > $out/et_kdd12.txt 2>&1
timeout -k 10 200 python tools/epoch_times.py kkbox 25 > $out/et_kkbox.txt 2>&1
timeout -k 10 200 python tools/epoch_times.py outbrain 25 > $out/et_ob.txt 2>&1
paste $out/et_kdd12.txt $out/et_kkbox.txt $out/et_ob.txt
for cfg in "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_tauq.so" "X=1"; do
  env $cfg timeout -k 10 200 python tools/profile_epoch.py fp32 2 outbrain > $out/pe_aa.txt 2>&1
  echo "== $cfg"; grep -E "epoch wall|hs_cross|feat_hv" $out/pe_aa.txt | head -4
done
