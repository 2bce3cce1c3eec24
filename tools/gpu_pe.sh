#!/bin/bash
# Per-family / per-half epoch breakdown for env configurations (repo root, GPU box):
#   bash tools/gpu_pe.sh <tag> "ENV=a" "ENV=b" ...   (fp32 kkbox, epochs 3..6 after 2 warm-up)
set -e -o pipefail
tag=$1
shift
out=gpurun_out
mkdir -p $out
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python tools/profile_epoch.py fp32 4 > $out/pe_${tag}_$i.txt 2>&1
  echo "== $cfg"; head -40 $out/pe_${tag}_$i.txt
done
