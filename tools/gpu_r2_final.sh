#!/bin/bash
# Round-2 final check of the HEAD build: smoke, GPU tests, bench line, PMC passes of the
# bench (profiles/<tag>_bench_pmc.json), the config-5 workload at full size on one GPU,
# and one measurement per BASELINE config (tools/bench_configs.py).
# Usage: bash tools/gpu_r2_final.sh <tag>
tag=${1:-r2n}
bash tools/gpu_r2e.sh $tag || exit $?
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-1500
  if [ $rc -ne 0 ]; then tail -8 "gpurun_out/$name.log"; echo "[$name] fatal rc=$rc, stopping"; exit $rc; fi
}
run ${tag}_bench_complex_light 240 python -u bench.py --workload complex_light --steps 2 --warmup 1
run ${tag}_configs 600 python -u tools/bench_configs.py --out gpurun_out/${tag}_configs.json
