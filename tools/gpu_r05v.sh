#!/bin/bash
# Round-5 GPU step V: the entering pass scatters e into the partner's
# orientation (OCFFM_YTSC, default) against the in-block gather through perm
# (OCFFM_YTSC=0): the suite, then A/B at kkbox shape.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/r05v_pytest.log 2>&1 || { tail -40 $out/r05v_pytest.log; exit 1; }
tail -1 $out/r05v_pytest.log
bash tools/ab.sh 3 "X=1" "OCFFM_YTSC=0"
for cfg in "X=1" "OCFFM_YTSC=0"; do
  env $cfg timeout -k 10 200 python tools/profile_epoch.py fp32 2 > $out/pe_v.txt 2>&1
  echo "== $cfg"; grep -E "epoch wall|gd_cross_row|refresh_base|flush" $out/pe_v.txt | head -5
done
