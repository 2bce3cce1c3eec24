#!/bin/bash
# Round-5 GPU step Y: the CG direction pre-pass gated at >= 8 node
# references per column (config 5's user halves): the suite, then config-5
# per-family times with OCFFM_DIRPRE=0 / default (2 M rows), then the
# full-size config-5 shard through bench.py's cfg5 mode, both settings.
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/r05y_pytest.log 2>&1 || { tail -40 $out/r05y_pytest.log; exit 1; }
tail -1 $out/r05y_pytest.log
for cfg in "X=1" "OCFFM_DIRPRE=0"; do
  env $cfg timeout -k 10 300 python tools/profile_epoch.py fp32 2 cfg5 > $out/pe_y_${cfg:0:1}.txt 2>&1
  echo "== cfg5 $cfg"; grep -E "epoch wall|hs_cross|cg_dir|feat_hv|hs_side|aggregates|rows_T" $out/pe_y_${cfg:0:1}.txt | head -8
done
for cfg in "X=1" "OCFFM_DIRPRE=0"; do
  env $cfg timeout -k 10 400 python bench.py --steps 2 --warmup 1 --cpu-baseline off --sgd off > $out/r05y_bench_${cfg:0:1}.json 2> $out/r05y_bench_${cfg:0:1}.err
  python - $out/r05y_bench_${cfg:0:1}.json "$cfg" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
m = d.get("modes", {})
print(sys.argv[2], {k: (v.get("value"), v.get("ms_per_step")) for k, v in m.items() if isinstance(v, dict)})
PY
done
