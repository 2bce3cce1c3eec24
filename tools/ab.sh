#!/bin/bash
# A/B epoch time of env configurations, alternated R rounds (run from the repo root):
#   bash tools/ab.sh R "VAR=a VAR2=b" "VAR=c" ...
# Each run: bench.py --steps 10 --warmup 2, no CPU baseline, no SGD mode (AB_ARGS: more bench flags, e.g. --precision fp64).
set -e -o pipefail
rounds=$1
shift
out=gpurun_out
mkdir -p $out
: > $out/ab.txt
for r in $(seq 1 $rounds); do
  for cfg in "$@"; do
    env $cfg timeout -k 10 120 python bench.py --steps 10 --warmup 2 --cpu-baseline off --modes off --sgd off ${AB_ARGS:-} > $out/ab.json 2> $out/ab.err
    python - "$cfg" >> $out/ab.txt <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[1]:60s} ms/epoch {d['ms_per_step']:.3f}  cg {d['config']['cg_iters_per_epoch']}  {r['kernel']} {r['avg_launch_us']}us frac {r['frac']}")
PY
    tail -1 $out/ab.txt
  done
done
