#!/bin/bash
# SGD-mode bench line + rocprofv3 kernel stats of the same command (GPU box).
set -e -o pipefail
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_sgd.py > $out/bench_sgd.json 2> $out/bench_sgd.err
rm -rf $out/prof_sgd
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_sgd -o run \
  -- python tools/bench_sgd.py --cpu-sample 1000 > $out/prof_sgd.log 2>&1
cat $out/bench_sgd.json
find $out/prof_sgd -name '*kernel_stats.csv' -exec head -5 {} \;
