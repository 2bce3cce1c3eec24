#!/bin/bash
# Round-5 GPU step A (run from the repo root on the GPU box): the new
# multi-rank / full-size tests, the 8-rank rehearsal of bench.py on one GPU,
# and the driver's bench command with every mode.
set -e -o pipefail
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "n_ranks or configs_full" > $out/r05a_pytest.log 2>&1
tail -3 $out/r05a_pytest.log
OCFFM_BENCH_REHEARSAL=1 timeout -k 10 600 python bench.py --gpus 8 --steps 2 --warmup 1 \
  > $out/r05a_rehearsal8.json 2> $out/r05a_rehearsal8.err
cat $out/r05a_rehearsal8.json
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/r05a_bench.json 2> $out/r05a_bench.err
cat $out/r05a_bench.json
