#!/bin/bash
# complex_light_room (GPU preset, matrix-core filter) at 512^2 x 1024 spp: spp_split A/B
# (64 lanes per pixel turns sample stealing on: its LDS fits).
tag=${1:-r2r}
mkdir -p gpurun_out/$tag
for s in 8 16 32 64; do
  timeout -k 10 150 python -u bench.py --workload complex_light --width 512 --height 512 --spp 1024 --spp-split $s --steps 2 --warmup 1 --cpu-seconds 0 --no-parity > gpurun_out/$tag/split_$s.log 2>&1 || { tail -5 gpurun_out/$tag/split_$s.log; exit 1; }
  echo "split $s: $(tail -1 gpurun_out/$tag/split_$s.log | cut -c1-200)"
done
