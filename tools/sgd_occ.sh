set -e -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_sgd.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_sgd.log 2>&1
tail -1 gpurun_out/pt_sgd.log
for o in 1 0; do OCFFM_SGD_OCC=$o timeout -k 10 300 python tools/bench_sgd.py --cpu-sample 10 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('occ4' if '$o'=='1' else 'occ-auto', d['value'], d['ms_per_step'], d['roofline']['frac'])"; done
