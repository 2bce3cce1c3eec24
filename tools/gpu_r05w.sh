#!/bin/bash
# Round-5 GPU step W: the fused cross Hessian-vector step of id-like fields
# (k_hs_cross_fused; OCFFM_XFUSE=0: row pass + feature pass): the suite, then
# A/B fp32 and fp64 at kkbox shape, and per-family times.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "epochs or variants or kkbox_small or speculative or bit_identical" --timeout 300 --timeout-method thread \
  > $out/r05w_pytest.log 2>&1 || { tail -40 $out/r05w_pytest.log; exit 1; }
tail -1 $out/r05w_pytest.log
bash tools/ab.sh 3 "X=1" "OCFFM_XFUSE=0"
bash tools/ab64.sh 1 "X=1" "OCFFM_XFUSE=0"
for cfg in "X=1" "OCFFM_XFUSE=0"; do
  env $cfg timeout -k 10 200 python tools/profile_epoch.py fp32 2 > $out/pe_w.txt 2>&1
  echo "== $cfg"; grep -E "epoch wall|hs_cross|feat_hv" $out/pe_w.txt | head -5
done
