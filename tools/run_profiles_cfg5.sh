#!/bin/bash
# Config-5 profile collection on the GPU box (run from the repo root):
#   bash tools/run_profiles_cfg5.sh <tag>
# 1. rocprofv3 --kernel-trace --stats of two config-5 epochs (2 M rows, k=64)
# 2. separate --pmc FETCH_SIZE / WRITE_SIZE passes over one epoch (MI355X
#    guide: they do not fit one pass), summarised per kernel family by
#    tools/pmc_summary.py into gpurun_out/summ_<tag>/ (copied to profiles/).
set -e -o pipefail
tag=${1:-r03_cfg5}
out=gpurun_out
sm=$out/summ_$tag
mkdir -p $out $sm
export TMPDIR=/tmp
P="python tools/profile_epoch.py fp32 1 cfg5"
rm -rf $out/prof_$tag $out/pmcf_$tag $out/pmcw_$tag
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_$tag -o run -- $P > $out/prof_$tag.log 2>&1
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmcf_$tag -o run -- $P > $out/pmcf_$tag.log 2>&1
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmcw_$tag -o run -- $P > $out/pmcw_$tag.log 2>&1
f() { find $1 -name "$2" | head -1; }
cp $(f $out/prof_$tag '*kernel_stats.csv') $sm/${tag}_kernel_stats.csv
python tools/pmc_summary.py stats $sm/${tag}_kernel_stats.csv $sm/${tag}_kernel_stats.json > $sm/stats.txt
python tools/pmc_summary.py traffic $(f $out/pmcf_$tag '*counter_collection.csv') $(f $out/pmcw_$tag '*counter_collection.csv') \
  $sm/${tag}_pmc_traffic.json > $sm/traffic.txt
cat $sm/*.txt
