#!/bin/bash
# Round-5 GPU step K: column-block pass gate (outbrain), fp64 gather-width A/B.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "heavy or variants_fp64 or execution or configs_full or two_ranks or n_ranks" > $out/r05k_pytest.log 2>&1 \
  || { tail -40 $out/r05k_pytest.log; exit 1; }
tail -2 $out/r05k_pytest.log
timeout -k 10 200 python tools/profile_epoch.py fp32 2 outbrain > $out/pe_ob.txt 2>&1
head -14 $out/pe_ob.txt
timeout -k 10 200 python tools/profile_epoch.py fp32 2 kdd12 > $out/pe_kdd.txt 2>&1
head -14 $out/pe_kdd.txt
bash tools/ab64.sh 2 "OCFFM_X=0" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_hs16.so" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_gd8.so"
cp $out/ab64.txt $out/r05k_ab64.txt
