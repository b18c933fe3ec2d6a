#!/bin/bash
# Per-config measurements (tools/bench_configs.py, one process per config so output keeps
# flowing) and a bench line that picks up the committed PMC profile of this build.
# Usage: bash tools/gpu_r2_configs.sh <tag>
tag=${1:-r2o}
mkdir -p gpurun_out/$tag
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$tag/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -1 "gpurun_out/$tag/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then tail -8 "gpurun_out/$tag/$name.log"; echo "[$name] fatal rc=$rc, stopping"; exit $rc; fi
}
run bench 300 python -u bench.py --steps 20 --warmup 3
for c in c1 c2 c3 c4 c5; do
  run cfg_$c 170 python -u tools/bench_configs.py --only $c --cpu --out gpurun_out/$tag/configs_$c.json
done
for c in c3 c4 c5; do
  run cpu_$c 170 python -u tools/bench_configs.py --only none --cpu $c --out gpurun_out/$tag/cpu_$c.json
done
