#!/bin/bash
# GPU session: GPU tests of the default build, then in-process A/B of build variants
# (Cornell 512^2/256 spp at spp_split 64 and 8).  Usage: bash tools/gpu_ab_only.sh tag v1 v2 ...
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/${tag}_pytest_gpu.log; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
V=""; for v in "$@"; do V="$V build/variants/$v"; done
timeout -k 10 240 python -u tools/ab_render.py $V --rounds 5 --split 64 > gpurun_out/${tag}_ab64.log 2>&1 || exit $?
tail -1 gpurun_out/${tag}_ab64.log
