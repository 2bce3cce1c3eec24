#!/bin/bash
# Round-5 GPU step C: the suite with the persistent column-Gram CG on, then
# A/B runs (fp32: persistent CG on/off; fp64: wide lanes / VALU T builds).
set -e -o pipefail
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/r05c_pytest.log 2>&1 || { tail -30 $out/r05c_pytest.log; exit 1; }
tail -3 $out/r05c_pytest.log
bash tools/ab.sh 2 "OCFFM_CGP=0" "OCFFM_CGP=1" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_notm.so"
cp $out/ab.txt $out/r05c_ab.txt
bash tools/ab64.sh 2 "OCFFM_CGP=0" "OCFFM_CGP=1" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_f64w.so" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_notm.so"
cp $out/ab64.txt $out/r05c_ab64.txt
