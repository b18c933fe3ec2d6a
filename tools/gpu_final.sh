#!/bin/bash
# round-end check of the current build: GPU tests, smoke (run with: bash tools/gpu_final.sh <tag>)
set -o pipefail
tag=${1:-r2b}
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/${tag}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${tag}_smoke.log 2>&1 || { tail gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
