#!/bin/bash
# GPU session: parity tests of the default build, then in-process A/B of variants
# on both presets.  Usage: bash tools/gpu_ab.sh variant1 variant2 ...
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
V=""; for v in "$@"; do V="$V build/variants/$v"; done
timeout -k 10 300 python tools/ab_render.py $V --rounds 5 > gpurun_out/ab.log 2>&1 || exit $?
tail -1 gpurun_out/ab.log
timeout -k 10 300 python tools/ab_render.py $V --rounds 3 --preset 1 > gpurun_out/ab_gpu.log 2>&1 || exit $?
tail -1 gpurun_out/ab_gpu.log
