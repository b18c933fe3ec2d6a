#!/bin/bash
# One GPU session: smoke, gpu tests, bench.  Every GPU step has its own time
# limit; a step that faults, aborts, segfaults or times out ends the session
# (exit codes other than 0 = pass and 1 = test failures).
mkdir -p gpurun_out
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[$name] fatal rc=$rc, stopping"; exit $rc; fi
  return 0
}
run smoke 150 python -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 600 python -m pytest tests -q -m gpu
run bench 240 python bench.py --steps 10 --warmup 2
run bench_sarsa 240 python tools/bench_sarsa.py --frames 4
