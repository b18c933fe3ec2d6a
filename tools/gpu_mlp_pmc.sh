#!/bin/bash
# PMC passes over the standalone DQN forward (tools/bench_dqn.py --no-render).
tag=${1:-mlp_pmc}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/$tag; mkdir -p $out
RUN="python3 tools/bench_dqn.py --scene archway --no-render"
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d $out/$name -o $name --output-format csv -- $RUN > $out/$name.log 2>&1
  local rc=$?; echo "[$name] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/$name.log; exit $rc; fi
}
pass m1 SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
pass m2 SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_WAVES
pass m3 TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
