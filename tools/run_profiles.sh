#!/bin/bash
# Round profile collection on the GPU box (run from the repo root):
#   bash tools/run_profiles.sh <tag>
# 1. bench.py (default config) -> gpurun_out/bench_<tag>.json
# 2. rocprofv3 --kernel-trace --stats of the same bench command
# 3. separate --pmc FETCH_SIZE / WRITE_SIZE passes (MI355X guide: they do
#    not fit one pass), summarised per kernel family by tools/pmc_summary.py.
set -e -o pipefail
tag=${1:-r01}
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $out/bench_$tag.json 2> $out/bench_$tag.err
rm -rf $out/prof_$tag $out/pmcf_$tag $out/pmcw_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_$tag -o run \
  -- python bench.py --steps 5 --warmup 2 --cpu-baseline off > $out/prof_$tag.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmcf_$tag -o run \
  -- python bench.py --steps 1 --warmup 1 --cpu-baseline off > $out/pmcf_$tag.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmcw_$tag -o run \
  -- python bench.py --steps 1 --warmup 1 --cpu-baseline off > $out/pmcw_$tag.log 2>&1
ls -R $out/prof_$tag $out/pmcf_$tag $out/pmcw_$tag | head -40
