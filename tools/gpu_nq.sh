#!/bin/bash
# Neural-Q renderer + training step: tests and the step benchmark
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_neuralq.py tests/test_dqn.py -k "neuralq or NeuralQ or explore or stats_epsilon or deterministic or door_room_obj or train or td" > gpurun_out/nq_tests.log 2>&1 || { tail -40 gpurun_out/nq_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/nq_tests.log | tail -12
timeout -k 10 200 python -u tools/bench_train.py > gpurun_out/train3.json 2> gpurun_out/train3.err || { tail gpurun_out/train3.err; exit 1; }
cat gpurun_out/train3.json
