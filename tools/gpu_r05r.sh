#!/bin/bash
# Round-5 GPU step R: sg_bcast at 16 lanes per row by DPP row_newbcast (k = 64
# fp32) instead of ds_bpermute: the suite, then per-kernel times against the
# previous build (exp/libocffm_base.so), outbrain and config-5 shapes.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/r05r_pytest.log 2>&1 || { tail -40 $out/r05r_pytest.log; exit 1; }
tail -1 $out/r05r_pytest.log
for shape in outbrain cfg5; do
  for cfg in "X=1" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_base.so"; do
    env $cfg timeout -k 10 300 python tools/profile_epoch.py fp32 2 $shape > $out/pe_r_${shape}_${cfg:0:1}.txt 2>&1
    echo "== $shape $cfg"; head -12 $out/pe_r_${shape}_${cfg:0:1}.txt | grep -v amdgpu.ids
  done
done
