#!/bin/bash
# Round-4 profile collection on the GPU box (run from the repo root):
#   bash tools/run_profiles_r04.sh <tag> [kkbox|fp64|cfg5]...
# Per workload: rocprofv3 --kernel-trace --stats of a short bench run, then
# separate --pmc FETCH_SIZE / WRITE_SIZE passes (MI355X guide §HBM: they do
# not fit one pass), summarised per kernel family by tools/pmc_summary.py
# into gpurun_out/summ_<tag>/ (copied to profiles/ by hand).
#   kkbox : the headline (f32, kkbox shape, k=32)
#   fp64  : the same epochs in fp64 (the parity mode: modes.fp64's roofline)
#   cfg5  : the config-5 shard (modes.cfg5), CFG5_ROWS rows (default 12.5 M)
set -e -o pipefail
tag=${1:-r04}
shift || true
what=${@:-kkbox fp64}
out=gpurun_out
sm=$out/summ_$tag
mkdir -p $out $sm
export TMPDIR=/tmp
f() { find $1 -name "$2" | head -1; }
for w in $what; do
  case $w in
    kkbox) B="python bench.py --steps 5 --warmup 2 --cpu-baseline off --modes off --sgd off"
           P="python bench.py --steps 1 --warmup 1 --cpu-baseline off --modes off --sgd off"; pre=""; T=300;;
    fp64)  B="python bench.py --precision fp64 --steps 5 --warmup 2 --cpu-baseline off --modes off --sgd off"
           P="python bench.py --precision fp64 --steps 1 --warmup 1 --cpu-baseline off --modes off --sgd off"; pre="fp64_"; T=300;;
    cfg5)  export CFG5_ROWS=${CFG5_ROWS:-12500000}; B="python tools/profile_epoch.py fp32 1 cfg5"
           P="$B"; pre="cfg5_"; T=600;;
  esac
  rm -rf $out/prof_${tag}_$w $out/pmcf_${tag}_$w $out/pmcw_${tag}_$w
  timeout -k 10 $T rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_${tag}_$w -o run -- $B \
    > $out/prof_${tag}_$w.log 2>&1
  timeout -k 10 $T rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmcf_${tag}_$w -o run -- $P \
    > $out/pmcf_${tag}_$w.log 2>&1
  timeout -k 10 $T rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmcw_${tag}_$w -o run -- $P \
    > $out/pmcw_${tag}_$w.log 2>&1
  cp $(f $out/prof_${tag}_$w '*kernel_stats.csv') $sm/${tag}_${pre}kernel_stats.csv
  python tools/pmc_summary.py stats $sm/${tag}_${pre}kernel_stats.csv $sm/${tag}_${pre}kernel_stats.json \
    > $sm/${pre}stats.txt
  python tools/pmc_summary.py traffic $(f $out/pmcf_${tag}_$w '*counter_collection.csv') \
    $(f $out/pmcw_${tag}_$w '*counter_collection.csv') $sm/${tag}_${pre}pmc_traffic.json > $sm/${pre}traffic.txt
done
ls $sm
