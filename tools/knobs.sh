#!/bin/bash
# Epoch time under solver knobs (env), one bench line each (no CPU baseline).
set -e -o pipefail
out=gpurun_out
mkdir -p $out
: > $out/knobs.txt
for cfg in "$@"; do
  env $cfg timeout -k 10 120 python bench.py --steps 5 --warmup 2 --cpu-baseline off > $out/knob.json 2>$out/knob.err
  python - "$cfg" >> $out/knobs.txt <<'PY'
import json, sys
d = json.loads(open("gpurun_out/knob.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:40s} ms/epoch {d['ms_per_step']:.3f}  cg {d['config']['cg_iters_per_epoch']}  {d['roofline']['kernel']} {d['roofline']['avg_launch_us']}us")
PY
done
cat $out/knobs.txt
