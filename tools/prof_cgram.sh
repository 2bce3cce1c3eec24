set -e -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/pcg1 gpurun_out/pcg0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pcg1 -o run -- python bench.py --steps 5 --warmup 2 --cpu-baseline off > gpurun_out/pcg1.log 2>&1
OCFFM_CGRAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pcg0 -o run -- python bench.py --steps 5 --warmup 2 --cpu-baseline off > gpurun_out/pcg0.log 2>&1
for d in pcg1 pcg0; do find gpurun_out/$d -name '*kernel_stats.csv' -exec cp {} gpurun_out/$d.stats.csv \; ; done
