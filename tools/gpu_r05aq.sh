#!/bin/bash
# Round-5 GPU step AQ: fp64 segments of 48 positives by default: the suite,
# smoke(), then fp64 A/B against 32.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/r05aq_pytest.log 2>&1 || { tail -40 $out/r05aq_pytest.log; exit 1; }
tail -1 $out/r05aq_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
bash tools/ab64.sh 2 "X=1" "OCFFM_SEG_LEN=32"
