#!/bin/bash
# Round-5 GPU step AR: the driver's bench command on the final build.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/r05ar_bench.json 2> $out/r05ar_bench.err
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05ar_bench.json").read().strip().splitlines()[-1])
print("headline", d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["avg_launch_us"], d["roofline"]["frac"])
for k, v in d["modes"].items():
    print(k, v.get("value"), v.get("ms_per_step"))
PY
