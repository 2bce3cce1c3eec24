#!/bin/bash
# Round-5 GPU step H: the suite, then A/B of the column-block feature pass
# and the pair Grams, and the gd_cross gather probe's per-half profile.
set -e -o pipefail
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/r05h_pytest.log 2>&1 || { tail -40 $out/r05h_pytest.log; exit 1; }
tail -3 $out/r05h_pytest.log
bash tools/ab.sh 2 "OCFFM_FEATCOL=0 OCFFM_PGRAM=0" "OCFFM_PGRAM=0" "OCFFM_X=1"
cp $out/ab.txt $out/r05h_ab.txt
OCFFM_LIB=one-class-ffm_amd/exp/libocffm_probe.so timeout -k 10 200 python tools/profile_epoch.py fp32 4 > $out/pe_probe.txt 2>&1
grep -E "gd_|epoch wall" $out/pe_probe.txt
timeout -k 10 200 python tools/profile_epoch.py fp32 4 > $out/pe_h.txt 2>&1
head -30 $out/pe_h.txt
