#!/bin/bash
# bench.py's multi-rank flow (torchrun, 2 ranks) on a one-GPU box: both ranks
# on device 0, all-reduces through gloo (OCFFM_BENCH_REHEARSAL=1).
set -e -o pipefail
OCFFM_BENCH_REHEARSAL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/rehearsal.json 2> gpurun_out/rehearsal.err
cat gpurun_out/rehearsal.json
