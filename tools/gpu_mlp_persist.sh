#!/bin/bash
# k_dqn_mlp persistent (RT_MLP_PERSIST=1, a switch of the r2s experiment since removed from
# the source: DESIGN.md §4) vs one tile per workgroup (base): DQN tests on
# both builds, then the 1 M-ray forward and the archway 1024^2 x 4 spp render, interleaved.
tag=${1:-r2s}
mkdir -p gpurun_out/$tag
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$tag/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(tail -1 gpurun_out/$tag/$name.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then tail -20 "gpurun_out/$tag/$name.log"; echo "[$name] fatal rc=$rc, stopping"; exit $rc; fi
}
V=reinforcement-light-rays-pathtracer_amd/build/variants
for v in base persist; do
  RTMI_LIB=$V/$v/librtmi.so run tests_$v 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_dqn.py tests/test_neuralq.py
done
for r in 1 2; do
  for v in base persist; do
    RTMI_LIB=$V/$v/librtmi.so run dqn_${v}_$r 200 python -u tools/bench_dqn.py --spp 4 --steps 2
  done
done
