#!/bin/bash
# Round-5 GPU step AN: the multi-rank tests and the 8-rank rehearsal (x4)
# without the persistent CG kernel on the shared GPU.
out=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_dist.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/r05an_pytest.log 2>&1 || { tail -30 $out/r05an_pytest.log; exit 1; }
tail -1 $out/r05an_pytest.log
for i in 1 2 3 4; do
  OCFFM_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 8 --steps 2 --warmup 1 > $out/r05an_$i.json 2> $out/r05an_$i.err
  echo "run $i rc=$?"; grep -h "OcffmError" $out/r05an_$i.err | head -2
done
cut -c1-300 $out/r05an_1.json
