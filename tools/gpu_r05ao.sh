#!/bin/bash
# Round-5 GPU step AO: the whole GPU suite and smoke() on the final build.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/r05ao_pytest.log 2>&1 || { tail -40 $out/r05ao_pytest.log; exit 1; }
tail -1 $out/r05ao_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
