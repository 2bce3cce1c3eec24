#!/bin/bash
# Round-5 GPU step AE: resident-wave grids for the gradient and feature
# passes: the suite, then OCFFM_FEAT_FILL=0 / OCFFM_GD_FILL=0 A/B, fp32 + fp64.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/r05ae_pytest.log 2>&1 || { tail -40 $out/r05ae_pytest.log; exit 1; }
tail -1 $out/r05ae_pytest.log
bash tools/ab.sh 2 "X=1" "OCFFM_FEAT_FILL=0" "OCFFM_FEAT_FILL=0 OCFFM_GD_FILL=0"
bash tools/ab64.sh 2 "X=1" "OCFFM_FEAT_FILL=0" "OCFFM_FEAT_FILL=0 OCFFM_GD_FILL=0"
