#!/bin/bash
# Neural-Q training: tests, then the step benchmark and its kernel split
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_dqn.py -k "train or adam or td or learn or trainer" > gpurun_out/train2_tests.log 2>&1 || { tail -30 gpurun_out/train2_tests.log; exit 1; }
tail -2 gpurun_out/train2_tests.log
timeout -k 10 200 python -u tools/bench_train.py > gpurun_out/train2.json 2> gpurun_out/train2.err || { tail gpurun_out/train2.err; exit 1; }
cat gpurun_out/train2.json
bash tools/gpu_train_prof.sh train2_prof
