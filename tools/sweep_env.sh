#!/bin/bash
# Bench sweep over one environment knob (run from the repo root):
#   bash tools/sweep_env.sh VAR "v1 v2 ..." [steps]
# Prints ms/step, the dominant kernel and its average launch time per value.
set -e -o pipefail
var=$1
vals=$2
steps=${3:-10}
mkdir -p gpurun_out
for v in $vals; do
  env $var=$v timeout -k 10 300 python bench.py --steps $steps --warmup 2 --cpu-baseline off --sgd off > gpurun_out/sweep_${var}_$(basename $v).json 2> gpurun_out/sweep_${var}_$(basename $v).err
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep_${var}_$(basename $v).json').read().strip().splitlines()[-1]); r=d['roofline']; print('$var=$v', d['ms_per_step'], 'ms/step', r['kernel'], r['avg_launch_us'], 'us', 'frac', r['frac'])"
done
