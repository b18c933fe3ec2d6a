#!/bin/bash
# Kernel trace + SQ/TA counters of the DQN renderer (archway 512^2, 1 spp).
tag=${1:-dqn_prof}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/$tag; mkdir -p $out
RUN="python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 1"
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 "$@" -d $out/$name -o $name --output-format csv -- $RUN > $out/$name.log 2>&1
  local rc=$?; echo "[$name] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/$name.log; exit $rc; fi
}
pass kt --kernel-trace --stats
pass sq --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace
pass ta --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --kernel-trace
