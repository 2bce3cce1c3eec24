#!/bin/bash
# Round-5 GPU step E: the whole suite on the defaults, then the driver's bench command.
set -e -o pipefail
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/r05e_pytest.log 2>&1 || { tail -30 $out/r05e_pytest.log; exit 1; }
tail -3 $out/r05e_pytest.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/r05e_bench.json 2> $out/r05e_bench.err
cat $out/r05e_bench.json
