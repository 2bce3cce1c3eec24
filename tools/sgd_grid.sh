#!/bin/bash
# SGD launch-grid sweep on the GPU box (OCFFM_SGD_GRID: blocks of 4 waves per
# epoch launch; 1024 = 4 waves/SIMD resident on 256 CUs at occupancy 4).
set -e -o pipefail
for g in ${GRIDS:-1024 2048 4096 8192 512}; do
  OCFFM_SGD_GRID=$g timeout -k 10 200 python tools/bench_sgd.py --cpu-sample 10 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('grid $g', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
