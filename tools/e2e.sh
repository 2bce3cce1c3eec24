#!/bin/bash
# End-to-end phases of the drop-in CLI on kkbox-shape files (GPU box).
set -e -o pipefail
out=gpurun_out
mkdir -p $out /tmp/kk
timeout -k 10 120 python -c "
import sys; sys.path.insert(0, 'one-class-ffm_amd')
import synth; synth.kkbox().write('/tmp/kk')"
OCFFM_TIMING=1 timeout -k 10 300 ./one-class-ffm_amd/train -k 32 -l 4 -w 0.0078125 -r -1 -t ${1:-10} --fp32 \
  -p /tmp/kk/kkbox.te.ffm -o /tmp/kk/model.txt /tmp/kk/kkbox.item.ffm /tmp/kk/kkbox.tr.ffm > $out/e2e.out 2> $out/e2e.err
cat $out/e2e.out $out/e2e.err
