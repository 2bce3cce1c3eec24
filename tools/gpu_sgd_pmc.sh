#!/bin/bash
set -e -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_sgd.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_sgd.log 2>&1
tail -1 gpurun_out/pt_sgd.log
timeout -k 10 300 python tools/bench_sgd.py --cpu-sample 1000
PMC_CMD="python tools/bench_sgd.py --steps 1 --warmup 0 --cpu-sample 10" bash tools/pmc_passes.sh sgd k_sgd > /dev/null
python tools/pmc_kernels.py $(find gpurun_out/pmc_sgd -name '*counter_collection.csv')
