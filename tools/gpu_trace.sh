#!/bin/bash
# Kernel trace of a short bench (no events in the timed region) for gap analysis.
set -e -o pipefail
tag=${1:-tr}
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
rm -rf $out/trace_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_$tag -o run \
  -- python bench.py --steps 3 --warmup 1 --cpu-baseline off > $out/trace_$tag.log 2>&1
f=$(find $out/trace_$tag -name '*kernel_trace.csv' | head -1)
python tools/trace_gaps.py $f 200 > $out/gaps_$tag.txt
python tools/trace_by_grid.py $f > $out/bygrid_$tag.txt
cat $out/gaps_$tag.txt
