#!/bin/bash
# Round-5 GPU step AM: the 8-rank rehearsal four times (a one-off
# verdict-publication failure in its kernel-timing pass: how often).
out=gpurun_out
export TMPDIR=/tmp
for i in 1 2 3 4 5 6; do
  OCFFM_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 8 --steps 2 --warmup 1 > $out/r05am_$i.json 2> $out/r05am_$i.err
  echo "run $i rc=$?"; grep -h "OcffmError" $out/r05am_$i.err | head -2
done
