#!/bin/bash
# Round-5 GPU step G: pair-Gram parity tests, per-half profile and A/B of OCFFM_PGRAM.
set -e -o pipefail
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "variants_fp64 or execution_variants or bit_identical or speculative or heavy" > $out/r05g_pytest.log 2>&1 \
  || { tail -40 $out/r05g_pytest.log; exit 1; }
tail -3 $out/r05g_pytest.log
OCFFM_PGRAM=1 timeout -k 10 200 python tools/profile_epoch.py fp32 4 > $out/pe_g.txt 2>&1
grep -E "half\(0,1\)|half\(1,1\)|pg_step|pair_gram|feat_hv|hs_side|epoch wall" $out/pe_g.txt
bash tools/ab.sh 3 "OCFFM_PGRAM=0" "OCFFM_PGRAM=1"
cp $out/ab.txt $out/r05g_ab.txt
