#!/bin/bash
# Round-5 GPU step F: pair-Gram parity tests, then A/B of OCFFM_PGRAM.
set -e -o pipefail
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "variants_fp64 or execution_variants or bit_identical or speculative or heavy" > $out/r05f_pytest.log 2>&1 \
  || { tail -40 $out/r05f_pytest.log; exit 1; }
tail -3 $out/r05f_pytest.log
bash tools/ab.sh 3 "OCFFM_PGRAM=0" "OCFFM_PGRAM=1"
cp $out/ab.txt $out/r05f_ab.txt
