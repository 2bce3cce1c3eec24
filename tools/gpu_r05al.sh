#!/bin/bash
# Round-5 GPU step AL: the 8-rank rehearsal with the resident-wave grids off,
# then on (bisecting a verdict-publication failure in its kernel-timing pass).
out=gpurun_out
export TMPDIR=/tmp
OCFFM_GD_FILL=0 OCFFM_FEAT_FILL=0 OCFFM_ROW_FILL=0 OCFFM_SIDE_FILL=0 OCFFM_MISC_FILL=0 OCFFM_BENCH_REHEARSAL=1 \
  timeout -k 10 400 python bench.py --gpus 8 --steps 2 --warmup 1 > $out/r05al_off.json 2> $out/r05al_off.err
echo "off rc=$?"; grep -h "OcffmError" $out/r05al_off.err | head -3
OCFFM_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 8 --steps 2 --warmup 1 > $out/r05al_on.json 2> $out/r05al_on.err
echo "on rc=$?"; grep -h "OcffmError" $out/r05al_on.err | head -3
