#!/bin/bash
# per-kernel times of the Neural-Q training step (65,536 rays)
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
tag=${1:-train_prof}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/$tag -o $tag -- python3 /root/repo/tools/bench_train.py --batch 65536 --steps 10 > /root/repo/gpurun_out/$tag.log 2>&1 || { tail -20 /root/repo/gpurun_out/$tag.log; exit 1; }
f=$(find /root/repo/gpurun_out/$tag -name "*kernel_stats.csv" | head -1)
cp $f /root/repo/gpurun_out/${tag}_kernel_stats.csv
cut -d, -f1-4 $f | head -25
