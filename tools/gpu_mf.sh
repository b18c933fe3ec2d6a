#!/bin/bash
# matrix-core filter: parity tests, then the bench line (run: bash tools/gpu_mf.sh <tag>)
set -o pipefail
tag=${1:-mf}
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mf_filter.py tests/test_gpu_parity.py tests/test_cull.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/${tag}_bench.log 2>&1 || { tail gpurun_out/${tag}_bench.log; exit 1; }
tail -2 gpurun_out/${tag}_bench.log
