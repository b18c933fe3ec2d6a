#!/bin/bash
# Round-2 check of the HEAD build: smoke, GPU tests, bench line, PMC passes of the bench.
# Usage: bash tools/gpu_r2e.sh <tag>
mkdir -p gpurun_out
tag=${1:-r2e}
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-2500
  if [ $rc -ne 0 ]; then tail -8 "gpurun_out/$name.log"; echo "[$name] fatal rc=$rc, stopping"; exit $rc; fi
}
run ${tag}_smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
run ${tag}_pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread
run ${tag}_bench 300 python -u bench.py --steps 20 --warmup 3
bash tools/gpu_bench_pmc.sh $tag > gpurun_out/${tag}_pmc.log 2>&1; echo "pmc rc=$?"
cat gpurun_out/${tag}_pmc.log | cut -c1-300
