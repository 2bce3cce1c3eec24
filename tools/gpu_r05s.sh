#!/bin/bash
# Round-5 GPU step S: SQ issue / wait counters per kernel (kkbox, outbrain),
# one rocprofv3 --pmc pass per counter set (<= 8 SQ counters each).
set -e -o pipefail
out=gpurun_out
export TMPDIR=/tmp
rocprofv3 -L > $out/r05s_counters.txt 2>&1 || true
A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR"
for w in kkbox outbrain; do
  if [ $w = kkbox ]; then P="python bench.py --steps 1 --warmup 1 --cpu-baseline off --modes off --sgd off"
  else P="python tools/profile_epoch.py fp32 1 outbrain"; fi
  for s in A B; do
    rm -rf $out/sq${s}_$w
    timeout -s KILL 240 rocprofv3 --pmc ${!s} --output-format csv -d $out/sq${s}_$w -o run -- $P > $out/sq${s}_$w.log 2>&1
  done
  python tools/pmc_kernels.py $(find $out/sqA_$w $out/sqB_$w -name '*counter_collection.csv') > $out/r05s_sq_$w.txt
  echo "== $w"; wc -l $out/r05s_sq_$w.txt
done
