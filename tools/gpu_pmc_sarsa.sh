#!/bin/bash
# PMC passes over one SARSA frame (door_room 512^2/256 spp), one rocprofv3 run each.
tag=${1:-sarsa_pmc}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/$tag; mkdir -p $out
RUN="python3 tools/bench_sarsa.py --frames 1"
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d $out/$name -o $name --output-format csv -- $RUN > $out/$name.log 2>&1
  local rc=$?; echo "[$name] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/$name.log; exit $rc; fi
}
[ -n "$ONLY_MEM" ] || {
pass sq1 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
pass sq2 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_RD
pass fetch FETCH_SIZE
pass tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum
}
pass tlb TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum
pass ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
pass sq3 SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE
