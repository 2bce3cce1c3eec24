#!/bin/bash
# Profile collection on the GPU box (run from the repo root):
#   bash tools/run_profiles.sh <tag> [kkbox|fp64|cfg5|kdd12|outbrain|sgd]...
# Per workload: rocprofv3 --kernel-trace --stats of a short run, then
# separate --pmc FETCH_SIZE / WRITE_SIZE passes (MI355X guide §HBM: they do
# not fit one pass), summarised per kernel family (and, for the positive
# gather kernels, per template instantiation) by tools/pmc_summary.py into
# gpurun_out/summ_<tag>/ (copied to profiles/ by hand).
set -e -o pipefail
tag=${1:-r06}
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
    sgd)   B="python tools/bench_sgd.py --steps 3 --warmup 1 --cpu-sample 0"; P="$B"; pre="sgd_"; T=300;;
    kdd12|outbrain) B="python tools/profile_epoch.py fp32 3 $w"; P="python tools/profile_epoch.py fp32 1 $w"
           pre="${w}_"; T=300;;
  esac
  rm -rf $out/prof_${tag}_$w $out/pmcf_${tag}_$w $out/pmcw_${tag}_$w
  timeout -k 10 $T rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_${tag}_$w -o run -- $B \
    > $out/prof_${tag}_$w.log 2>&1
  timeout -k 10 $T rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmcf_${tag}_$w -o run -- $P \
    > $out/pmcf_${tag}_$w.log 2>&1
  timeout -k 10 $T rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmcw_${tag}_$w -o run -- $P \
    > $out/pmcw_${tag}_$w.log 2>&1
  st=$(f $out/prof_${tag}_$w '*kernel_stats.csv')
  fc=$(f $out/pmcf_${tag}_$w '*counter_collection.csv')
  wc=$(f $out/pmcw_${tag}_$w '*counter_collection.csv')
  cp $st $sm/${tag}_${pre}kernel_stats.csv
  python tools/pmc_summary.py stats $st $sm/${tag}_${pre}kernel_stats.json > $sm/${pre}stats.txt
  python tools/pmc_summary.py traffic $fc $wc $sm/${tag}_${pre}pmc_traffic.json > $sm/${pre}traffic.txt
  python tools/pmc_summary.py variants $st $fc $wc "k_gd_cross_seg|k_hs_cross_seg" \
    $sm/${tag}_${pre}variants.json > $sm/${pre}variants.txt
  echo "== $w"; head -8 $sm/${pre}stats.txt; cat $sm/${pre}variants.txt
done
ls $sm
