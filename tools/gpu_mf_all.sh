#!/bin/bash
# Matrix-core filter in the GPU-preset, SARSA and DQN kernels: the whole GPU suite on the
# default build, then A/B against the fp32-filter build (mf0), interleaved rounds:
# complex_light_room 1024^2 x 64 spp, door_room SARSA frames, archway DQN 1024^2 x 4 spp.
# Usage: bash tools/gpu_mf_all.sh <tag>
tag=$1
mkdir -p gpurun_out/$tag
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$tag/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(tail -1 gpurun_out/$tag/$name.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then tail -30 "gpurun_out/$tag/$name.log"; echo "[$name] fatal rc=$rc, stopping"; exit $rc; fi
}
run pytest_gpu 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests
V=reinforcement-light-rays-pathtracer_amd/build/variants
for r in 1 2; do
  for v in mf0 mf; do
    RTMI_LIB=$V/$v/librtmi.so run cl_${v}_$r 200 python -u bench.py --workload complex_light --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 --cpu-seconds 0 --no-parity
    run sarsa_${v}_$r 200 python -u tools/bench_sarsa.py --frames 2 --lib build/variants/$v
    RTMI_LIB=$V/$v/librtmi.so run dqn_${v}_$r 200 python -u tools/bench_dqn.py --spp 4 --steps 2
  done
done
