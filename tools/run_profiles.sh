#!/bin/bash
# Round profile collection on the GPU box (run from the repo root):
#   bash tools/run_profiles.sh <tag>
# Newton-CG headline (bench.py) and SGD mode (tools/bench_sgd.py):
# 1. the bench line -> gpurun_out/bench_<tag>.json / bench_sgd_<tag>.json
# 2. rocprofv3 --kernel-trace --stats of the same command
# 3. separate --pmc FETCH_SIZE / WRITE_SIZE passes (MI355X guide: they do
#    not fit one pass), summarised per kernel family by tools/pmc_summary.py
#    into gpurun_out/summ_<tag>/ (copied to profiles/ by hand).
set -e -o pipefail
tag=${1:-r01}
out=gpurun_out
sm=$out/summ_$tag
mkdir -p $out $sm
export TMPDIR=/tmp
B="python bench.py --steps 5 --warmup 2 --cpu-baseline off --modes off --sgd off"
S="python tools/bench_sgd.py --steps 3 --warmup 1 --cpu-sample 10"
timeout -k 10 300 python bench.py > $out/bench_$tag.json 2> $out/bench_$tag.err
timeout -k 10 300 python tools/bench_sgd.py > $out/bench_sgd_$tag.json 2> $out/bench_sgd_$tag.err
rm -rf $out/prof_$tag $out/pmcf_$tag $out/pmcw_$tag $out/sprof_$tag $out/spmcf_$tag $out/spmcw_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_$tag -o run -- $B > $out/prof_$tag.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmcf_$tag -o run \
  -- python bench.py --steps 1 --warmup 1 --cpu-baseline off --modes off --sgd off > $out/pmcf_$tag.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmcw_$tag -o run \
  -- python bench.py --steps 1 --warmup 1 --cpu-baseline off --modes off --sgd off > $out/pmcw_$tag.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/sprof_$tag -o run -- $S > $out/sprof_$tag.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_sgd --output-format csv -d $out/spmcf_$tag -o run \
  -- python tools/bench_sgd.py --steps 1 --warmup 0 --cpu-sample 10 > $out/spmcf_$tag.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_sgd --output-format csv -d $out/spmcw_$tag -o run \
  -- python tools/bench_sgd.py --steps 1 --warmup 0 --cpu-sample 10 > $out/spmcw_$tag.log 2>&1
f() { find $1 -name "$2" | head -1; }
cp $(f $out/prof_$tag '*kernel_stats.csv') $sm/${tag}_kernel_stats.csv
cp $(f $out/sprof_$tag '*kernel_stats.csv') $sm/${tag}_sgd_kernel_stats.csv
python tools/pmc_summary.py stats $sm/${tag}_kernel_stats.csv $sm/${tag}_kernel_stats.json > $sm/stats.txt
python tools/pmc_summary.py stats $sm/${tag}_sgd_kernel_stats.csv $sm/${tag}_sgd_kernel_stats.json > $sm/sgd_stats.txt
python tools/pmc_summary.py traffic $(f $out/pmcf_$tag '*counter_collection.csv') $(f $out/pmcw_$tag '*counter_collection.csv') \
  $sm/${tag}_pmc_traffic.json > $sm/traffic.txt
python tools/pmc_summary.py traffic $(f $out/spmcf_$tag '*counter_collection.csv') $(f $out/spmcw_$tag '*counter_collection.csv') \
  $sm/${tag}_sgd_pmc_traffic.json > $sm/sgd_traffic.txt
cp $out/bench_$tag.json $sm/${tag}_bench.json
cp $out/bench_sgd_$tag.json $sm/${tag}_sgd_bench.json
cat $sm/*.txt $sm/*bench.json
