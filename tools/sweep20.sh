#!/bin/bash
# Epoch time of env configurations at the driver's command (--steps 20 --warmup 5),
# alternated R rounds (run from the repo root):  bash tools/sweep20.sh R "VAR=a" "VAR=b" ...
set -e -o pipefail
rounds=$1
shift
out=gpurun_out
mkdir -p $out
: > $out/sweep20.txt
for r in $(seq 1 $rounds); do
  for cfg in "$@"; do
    env $cfg timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-baseline off --modes off --sgd off \
      > $out/sweep20.json 2> $out/sweep20.err
    python - "$cfg" >> $out/sweep20.txt <<'PY'
import json, sys
d = json.loads(open("gpurun_out/sweep20.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:40s} ms/epoch {d['ms_per_step']:.3f} cg {d['config']['cg_iters_per_epoch']}")
PY
    tail -1 $out/sweep20.txt
  done
done
