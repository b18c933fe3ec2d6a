#!/bin/bash
# MFMA filter round 2: parity tests on the default build, then in-process A/B of variants
set -o pipefail
tag=${1:-mf2}
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mf_filter.py tests/test_gpu_parity.py tests/test_cull.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ab_render.py build/variants/nomf build/variants/mf_lds_w5 build/variants/coop_w4 build/variants/coop_w5 build/variants/coop_lds_w5 --split 64 --rounds 7 > gpurun_out/${tag}_ab.json 2>gpurun_out/${tag}_ab.err || { tail -5 gpurun_out/${tag}_ab.err; exit 1; }
cat gpurun_out/${tag}_ab.json
