#!/bin/bash
# GPU tests, A/B of render builds, default bench line, PMC profile of the bench workload.
mkdir -p gpurun_out
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-1500
  if [ $rc -ne 0 ]; then tail -8 "gpurun_out/$name.log"; echo "[$name] fatal rc=$rc, stopping"; exit $rc; fi
}
tag=$1; shift
run ${tag}_pytest 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread
if [ $# -gt 0 ]; then
  V=""; for v in "$@"; do V="$V build/variants/$v"; done
  run ${tag}_ab 240 python -u tools/ab_render.py $V --rounds 7 --split 64
fi
run ${tag}_bench 300 python -u bench.py --steps 20 --warmup 3
bash tools/gpu_bench_pmc.sh $tag > gpurun_out/${tag}_pmc.log 2>&1; echo "pmc rc=$?"
