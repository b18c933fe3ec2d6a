#!/bin/bash
# DQN tests + bench_dqn for each variant (separate processes, RTMI_LIB).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dqn.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_dqn.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_dqn.log; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
P=$PWD/reinforcement-light-rays-pathtracer_amd/build/variants
for v in "$@"; do
  for sc in archway door_room; do
    RTMI_LIB=$P/$v/librtmi.so timeout -k 10 240 python tools/bench_dqn.py --scene $sc --width 512 --spp 1 --steps 2 > gpurun_out/dqn_${v}_$sc.log 2>&1 || exit $?
    echo "$v $sc: $(tail -1 gpurun_out/dqn_${v}_$sc.log)"
  done
done
