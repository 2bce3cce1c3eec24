#!/bin/bash
# Round-5 GPU step D: the wide-fp64-lane build through the fp64 parity tests,
# then fp64 and fp32 A/B of the builds.
set -e -o pipefail
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
W=one-class-ffm_amd/exp/libocffm_f64w.so
N=one-class-ffm_amd/exp/libocffm_notm.so
OCFFM_LIB=$W timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "fp64 or heavy or execution or block_by_block" > $out/r05d_pytest_w.log 2>&1 \
  || { tail -30 $out/r05d_pytest_w.log; exit 1; }
tail -2 $out/r05d_pytest_w.log
bash tools/ab64.sh 2 "OCFFM_X=0" "OCFFM_LIB=$W" "OCFFM_LIB=$N"
cp $out/ab64.txt $out/r05d_ab64.txt
bash tools/ab.sh 2 "OCFFM_X=0" "OCFFM_LIB=$N" "OCFFM_CGP=0"
cp $out/ab.txt $out/r05d_ab.txt
