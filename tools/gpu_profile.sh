#!/bin/bash
# rocprofv3 passes over one bench run each: kernel trace + stats, then PMC
# counters in separate passes (FETCH_SIZE and WRITE_SIZE cannot share a pass).
# Usage: bash tools/gpu_profile.sh <tag> [bench args...]
tag=${1:-r1}; shift
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/prof_$tag
mkdir -p $out
BENCH="python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-parity $*"
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -3 "$out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[$name] fatal rc=$rc, stopping"; exit $rc; fi
}
step kt 300 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- $BENCH
rocprofv3 -L > $out/counters_list.txt 2>&1 || true
step fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/fetch -o fetch --output-format csv -- $BENCH
step write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $out/write -o write --output-format csv -- $BENCH
step sq 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace -d $out/sq -o sq --output-format csv -- $BENCH
# kernel statistics of the learned-sampling paths (configs 3 and 4)
step kt_sarsa 300 rocprofv3 --kernel-trace --stats -d $out/kt_sarsa -o kt_sarsa --output-format csv -- python3 tools/bench_sarsa.py --frames 2
step kt_dqn 300 rocprofv3 --kernel-trace --stats -d $out/kt_dqn -o kt_dqn --output-format csv -- python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 1
step fetch_dqn 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/fetch_dqn -o fetch_dqn --output-format csv -- python3 tools/bench_dqn.py --scene archway --width 256 --spp 1 --steps 1
# Neural-Q training step
step kt_train 300 rocprofv3 --kernel-trace --stats -d $out/kt_train -o kt_train --output-format csv -- python3 tools/bench_train.py --batch 4096 --steps 10
