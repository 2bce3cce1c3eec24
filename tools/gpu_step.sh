#!/bin/bash
# GPU box: run a list of pytest node ids / files (one process, per-test
# timeout), then optionally smoke and the bench.  Usage:
#   tools/gpu_step.sh TAG "pytest args" [smoke] [bench "bench args"]
set -e -o pipefail
tag=$1; shift
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
eval "timeout -k 10 900 python -u -m pytest $1 ${PYX--x} -v --timeout 300 --timeout-method thread" > $out/pytest_$tag.log 2>&1
shift
if [ "$1" = smoke ]; then
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke_$tag.log 2>&1
  shift
fi
if [ "$1" = bench ]; then
  timeout -k 10 600 python bench.py $2 > $out/bench_$tag.json 2> $out/bench_$tag.err
  cat $out/bench_$tag.json
fi
tail -3 $out/pytest_$tag.log
