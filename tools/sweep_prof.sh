#!/bin/bash
# Bench + rocprofv3 kernel stats over one environment knob (run from the repo root):
#   bash tools/sweep_prof.sh VAR "v1 v2 ..." "family1 family2"
# Prints ms/step and the average launch time of each named kernel family.
set -e -o pipefail
var=$1
vals=$2
fams=$3
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in $vals; do
  d=gpurun_out/sp_${var}_$(basename $v)
  rm -rf $d
  env $var=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
    python bench.py --steps 10 --warmup 2 --cpu-baseline off --sgd off > $d.json 2> $d.err
  python tools/pmc_summary.py stats $(find $d -name '*kernel_stats.csv' | head -1) $d/stats.json > $d/stats.txt
  ms=$(python -c "import json; print(json.loads(open('$d.json').read().strip().splitlines()[-1])['ms_per_step'])")
  line="$var=$v ms/step $ms"
  for f in $fams; do
    a=$(python -c "import json; d=json.load(open('$d/stats.json')); print(round(d.get('$f',{}).get('avg_us',0),1))")
    line="$line $f=$a"
  done
  echo $line
done
