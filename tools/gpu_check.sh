#!/bin/bash
# GPU box check: parity tests, smoke, one bench line (run from the repo root).
set -e -o pipefail
tag=${1:-chk}
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_$tag.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke_$tag.log 2>&1
timeout -k 10 300 python bench.py > $out/bench_$tag.json 2> $out/bench_$tag.err
cat $out/bench_$tag.json
