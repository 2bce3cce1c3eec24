#!/bin/bash
# A/B of fp64 epoch time across library builds / env settings, alternated R rounds:
#   bash tools/ab64.sh R "VAR=a" "OCFFM_LIB=one-class-ffm_amd/exp/libocffm_x.so" ...
set -e -o pipefail
rounds=$1
shift
out=gpurun_out
mkdir -p $out
: > $out/ab64.txt
for r in $(seq 1 $rounds); do
  for cfg in "$@"; do
    env $cfg timeout -k 10 150 python bench.py --precision fp64 --steps 10 --warmup 2 --cpu-baseline off --modes off \
      --sgd off > $out/ab64.json 2> $out/ab64.err
    python - "$cfg" >> $out/ab64.txt <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab64.json").read().strip().splitlines()[-1])
r = d["roofline"]
fam = r.get("families_ms_per_epoch", {})
print(f"{sys.argv[1]:55s} ms/epoch {d['ms_per_step']:.3f} cg {d['config']['cg_iters_per_epoch']} {r['kernel']} "
      f"{r['avg_launch_us']}us " + " ".join(f"{k}={v}" for k, v in list(fam.items())[:4]))
PY
    tail -1 $out/ab64.txt
  done
done
