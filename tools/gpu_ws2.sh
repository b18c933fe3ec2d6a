#!/bin/bash
# weight-stationary MLP A/B (after a change): parity test, then forward + render
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_dqn.py -k "stationary or forward or config4" > gpurun_out/ws2_tests.log 2>&1 || { tail -30 gpurun_out/ws2_tests.log; exit 1; }
tail -2 gpurun_out/ws2_tests.log
for k in stream stationary; do
  timeout -k 10 200 python -u tools/bench_dqn.py --mlp $k --spp 4 --steps 2 > gpurun_out/ws2_bench_$k.json 2>gpurun_out/ws2_bench_$k.err || exit 1
  cat gpurun_out/ws2_bench_$k.json
done
