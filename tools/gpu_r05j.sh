#!/bin/bash
# Round-5 GPU step J: profiles (kkbox, fp64, kdd12, outbrain) and the driver's bench line.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/r05j_bench.json 2> $out/r05j_bench.err
tail -c 3000 $out/r05j_bench.json
bash tools/run_profiles_r05.sh r05 kkbox fp64 kdd12 outbrain
