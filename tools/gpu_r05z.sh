#!/bin/bash
# Round-5 GPU step Z: the driver's bench command on the final build, then
# fresh profiles of the k = 64 / k = 16 shapes (row_newbcast changed them).
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/r05z_bench.json 2> $out/r05z_bench.err
cat $out/r05z_bench.json
bash tools/run_profiles_r05.sh r05f outbrain kdd12 cfg5 > $out/r05z_prof.log 2>&1
tail -30 $out/r05z_prof.log
