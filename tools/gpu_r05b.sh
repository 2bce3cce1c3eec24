#!/bin/bash
# Round-5 GPU step (run from the repo root on the GPU box): the whole GPU
# suite, an A/B of an experiment library against the default one, the
# 8-rank rehearsal of bench.py on one GPU, and the driver's bench command.
#   bash tools/gpu_r05b.sh <tag> [experiment .so for the A/B]
set -e -o pipefail
tag=${1:-r05b}
exp=${2:-}
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/${tag}_pytest.log 2>&1
tail -3 $out/${tag}_pytest.log
if [ -n "$exp" ]; then
  bash tools/ab.sh 2 "OCFFM_LIB=$exp" "OCFFM_X=0"
  cp $out/ab.txt $out/${tag}_ab.txt
fi
OCFFM_BENCH_REHEARSAL=1 timeout -k 10 600 python bench.py --gpus 8 --steps 2 --warmup 1 \
  > $out/${tag}_rehearsal8.json 2> $out/${tag}_rehearsal8.err
tail -c 600 $out/${tag}_rehearsal8.json
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/${tag}_bench.json 2> $out/${tag}_bench.err
cat $out/${tag}_bench.json
