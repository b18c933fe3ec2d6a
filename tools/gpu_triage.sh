#!/bin/bash
# Triage run: the whole GPU suite without -x (test failures do not stop the call; a crash,
# abort or timeout does), then the default bench line.
cd "$(dirname "$0")/.." || exit 1
out=gpurun_out/${1:-triage}; mkdir -p "$out"; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > "$out/tests.log" 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -30 "$out/tests.log"
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 3 > "$out/bench.log" 2>&1
rc=$?; echo "[bench] rc=$rc"; tail -3 "$out/bench.log"; exit $rc
