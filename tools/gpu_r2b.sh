#!/bin/bash
# Round-2 session: A/B of the render kernel builds, the bench line (default + the other
# BASELINE workloads at reduced spp), then the PMC profile of the default bench workload.
mkdir -p gpurun_out
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -1 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then tail -8 "gpurun_out/$name.log"; echo "[$name] fatal rc=$rc, stopping"; exit $rc; fi
}
if [ $# -gt 0 ]; then
  V=""; for v in "$@"; do V="$V build/variants/$v"; done
  run b_ab 240 python -u tools/ab_render.py $V --rounds 7 --split 64
fi
run b_bench 300 python -u bench.py --steps 20 --warmup 3
run b_sarsa 300 python -u bench.py --workload door_room_sarsa --steps 3 --warmup 1 --cpu-seconds 0
run b_dqn 300 python -u bench.py --workload archway_dqn --spp 8 --steps 2 --warmup 1 --cpu-seconds 0
run b_c5 300 python -u bench.py --workload complex_light --spp 16 --steps 2 --warmup 1 --cpu-seconds 0 --no-parity
bash tools/gpu_bench_pmc.sh r2b
