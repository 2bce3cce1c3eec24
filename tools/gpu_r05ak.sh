#!/bin/bash
# Round-5 GPU step AK: final-build profiles of the headline and fp64 shapes,
# smoke(), and the 8-rank rehearsal of bench.py on one GPU.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
bash tools/run_profiles_r05.sh r05g kkbox fp64 > $out/r05ak_prof.log 2>&1
tail -12 $out/r05ak_prof.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/r05ak_smoke.txt 2>&1
tail -3 $out/r05ak_smoke.txt
OCFFM_BENCH_REHEARSAL=1 timeout -k 10 600 python bench.py --gpus 8 --steps 2 --warmup 1 \
  > $out/r05ak_rehearsal8.json 2> $out/r05ak_rehearsal8.err
cut -c1-400 $out/r05ak_rehearsal8.json
