#!/bin/bash
# Round-5 GPU step N: next-segment staging in hs_cross (columns) and
# gd_cross (columns + stored values): parity subset, then per-kernel times
# against exp/libocffm_pf0.so (no gd_cross staging) and exp/libocffm_rs0.so
# (neither, nor the reduce-scatter), kkbox / kdd12 / outbrain shapes.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "gradient_and_hv or epochs_fp32 or variants_fp64 or kkbox_small or heavy" > $out/r05n_pytest.log 2>&1 \
  || { tail -40 $out/r05n_pytest.log; exit 1; }
tail -1 $out/r05n_pytest.log
bash tools/ab.sh 2 "X=1" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_pf0.so" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_rs0.so"
for shape in kkbox kdd12 outbrain; do
  for cfg in "X=1" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_pf0.so" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_rs0.so"; do
    env $cfg timeout -k 10 200 python tools/profile_epoch.py fp32 2 $shape > $out/pe_n.txt 2>&1
    echo "== $shape $cfg"; grep -E "epoch wall|hs_cross_row|gd_cross_row" $out/pe_n.txt | head -4
  done
done
