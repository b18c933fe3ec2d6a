#!/bin/bash
# SARSA GPU session: parity tests, then frame timings of the shipped build and A/B variants.
mkdir -p gpurun_out
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[$name] fatal rc=$rc, stopping"; exit $rc; fi
  return 0
}
run pytest_sarsa 400 python -m pytest tests/test_sarsa.py -q -m gpu
run bench_sarsa 200 python tools/bench_sarsa.py --frames 3
for v in "$@"; do
  run "bench_sarsa_$v" 200 python tools/bench_sarsa.py --frames 2 --lib "build/variants/$v"
done
