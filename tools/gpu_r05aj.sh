#!/bin/bash
# Round-5 GPU step AJ: the driver's bench command on the final build, then
# the config-5 MFMA grid sweep (tools/gpu_r05ai.sh).
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/r05aj_bench.json 2> $out/r05aj_bench.err
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05aj_bench.json").read().strip().splitlines()[-1])
print("headline", d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["avg_launch_us"], d["roofline"]["frac"])
for k, v in d["modes"].items():
    print(k, v.get("value"), v.get("ms_per_step"))
PY
bash tools/gpu_r05ai.sh
