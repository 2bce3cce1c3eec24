#!/bin/bash
# One GPU iteration (run from the repo root): parity tests, a short bench
# line (no CPU baseline, no SGD mode) and a rocprofv3 kernel trace of it.
#   bash tools/gpu_iter.sh <tag> [pytest -k expression]
set -e -o pipefail
tag=${1:-it}
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
if [ "$2" = "none" ]; then
  :
elif [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$2" > $out/pytest_$tag.log 2>&1
  tail -3 $out/pytest_$tag.log
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_$tag.log 2>&1
  tail -3 $out/pytest_$tag.log
fi
B="python bench.py --steps 10 --warmup 2 --cpu-baseline off --sgd off"
timeout -k 10 300 $B > $out/bench_$tag.json 2> $out/bench_$tag.err
cat $out/bench_$tag.json
rm -rf $out/prof_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_$tag -o run -- $B > $out/prof_$tag.log 2>&1
python tools/trace_by_grid.py $(find $out/prof_$tag -name '*kernel_trace.csv' | head -1) > $out/grid_$tag.txt; head -30 $out/grid_$tag.txt
