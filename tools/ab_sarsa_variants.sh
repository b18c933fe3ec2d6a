#!/bin/bash
# In-process-free A/B of librtmi variants on the config-3 frame (tools/bench_sarsa.py, frames 0-4
# at the bench's split 64), two interleaved rounds; logs under gpurun_out/<tag>/.
tag=$1; shift
mkdir -p gpurun_out/$tag
for r in 1 2; do for v in "$@"; do
  RTMI_LIB=reinforcement-light-rays-pathtracer_amd/build/variants/$v/librtmi.so timeout -k 10 150 python3 tools/bench_sarsa.py --split 64 --frames 5 > gpurun_out/$tag/${v}_$r.log 2>&1 || exit 1
  echo "$v $r $(tail -1 gpurun_out/$tag/${v}_$r.log | cut -c1-300)"
done; done
