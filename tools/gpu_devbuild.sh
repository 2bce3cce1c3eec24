#!/bin/bash
# Device data-layout build on the GPU box: its parity tests (and the full GPU
# suite with "all"), then the set-up phases (device vs host build) at kkbox
# and config-5 size.
set -e -o pipefail
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_devbuild.py -x -v --timeout 120 --timeout-method thread > $out/pytest_devbuild.log 2>&1
if [ "$1" = all ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_all.log 2>&1
fi
for w in kkbox cfg5; do
  OCFFM_TIMING=1 timeout -k 10 300 python tools/setup_timing.py $w > $out/setup_dev_$w.log 2>&1
  OCFFM_TIMING=1 OCFFM_HOST_BUILD=1 timeout -k 10 300 python tools/setup_timing.py $w > $out/setup_host_$w.log 2>&1
done
tail -2 $out/pytest_devbuild.log
for f in $out/setup_*.log; do echo "== $f"; grep -v amdgpu.ids $f; done
