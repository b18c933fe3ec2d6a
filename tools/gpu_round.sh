#!/bin/bash
# Full GPU session: parity tests, the default bench line, rocprofv3 profile passes.
# Usage: bash tools/gpu_round.sh <tag>
tag=${1:-r1}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$tag.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$tag.log
bash tools/gpu_profile.sh $tag
