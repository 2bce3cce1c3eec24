#!/bin/bash
# k_col_gram chunk-size sweep (OCFFM_CGRAM_CHUNK): rocprofv3 stats per size.
set -e -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in 64 128 256; do
  rm -rf gpurun_out/pch$c
  OCFFM_CGRAM_CHUNK=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pch$c -o run -- python bench.py --steps 5 --warmup 2 --cpu-baseline off > gpurun_out/pch$c.log 2>&1
  find gpurun_out/pch$c -name '*kernel_stats.csv' -exec cp {} gpurun_out/pch$c.stats.csv \;
done
