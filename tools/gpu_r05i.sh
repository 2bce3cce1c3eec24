#!/bin/bash
# Round-5 GPU step I: the suite, A/B of the segment processing order.
set -e -o pipefail
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/r05i_pytest.log 2>&1 || { tail -40 $out/r05i_pytest.log; exit 1; }
tail -3 $out/r05i_pytest.log
bash tools/ab.sh 3 "OCFFM_SORDER=0" "OCFFM_SORDER=1"
cp $out/ab.txt $out/r05i_ab.txt
timeout -k 10 200 python tools/profile_epoch.py fp32 4 > $out/pe_i.txt 2>&1
head -24 $out/pe_i.txt
