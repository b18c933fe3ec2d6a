#!/bin/bash
# weight-stationary MLP: parity, then forward + render A/B against the streaming kernel
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_dqn.py tests/test_facade.py tests/test_sarsa.py > gpurun_out/ws_tests.log 2>&1 || { tail -30 gpurun_out/ws_tests.log; exit 1; }
tail -2 gpurun_out/ws_tests.log
for k in stream stationary; do
  timeout -k 10 200 python -u tools/bench_dqn.py --mlp $k --spp 4 --steps 2 > gpurun_out/ws_bench_$k.json 2>gpurun_out/ws_bench_$k.err || exit 1
  cat gpurun_out/ws_bench_$k.json
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/ws_prof -o ws -- python3 /root/repo/tools/bench_dqn.py --spp 4 --steps 2 > /root/repo/gpurun_out/ws_prof.log 2>&1 || exit 1
find /root/repo/gpurun_out/ws_prof -name "*kernel_stats.csv" | head -1 | xargs head -8
cd /root/repo
timeout -k 10 200 python -u tools/bench_train.py > gpurun_out/train_mfma.json 2> gpurun_out/train_mfma.err || exit 1
cat gpurun_out/train_mfma.json
