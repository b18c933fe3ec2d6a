#!/bin/bash
# One GPU session: smoke, GPU tests, in-process A/B of build variants, bench line.
# Every GPU step runs under its own time limit; a fault, abort, segfault or time
# limit ends the session (exit codes other than 0 and 1).
# Usage: bash tools/gpu_session.sh <tag> [variant ...]
tag=${1:-s}; shift
mkdir -p gpurun_out
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/${tag}_$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -3 "gpurun_out/${tag}_$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[$name] fatal rc=$rc, stopping"; exit $rc; fi
  return 0
}
run smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread
if [ $# -gt 0 ]; then
  V=""; for v in "$@"; do V="$V build/variants/$v"; done
  run ab64 240 python -u tools/ab_render.py $V --rounds 5 --split 64
  run ab8 240 python -u tools/ab_render.py $V --rounds 3 --split 8
fi
run bench 300 python -u bench.py --steps 20 --warmup 3
