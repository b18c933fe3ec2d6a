#!/bin/bash
# SQ instruction-mix counters of the bench kernel, one rocprofv3 pass each.
# Usage: bash tools/gpu_pmc.sh <tag>
tag=${1:-pmc}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/$tag; mkdir -p $out
BENCH="python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-parity"
rocprofv3 -L > $out/counters_list.txt 2>&1 || true
pass() {  # name counters...
  local name=$1; shift
  for c in "$@"; do grep -q "\b$c\b" $out/counters_list.txt || { echo "skip $name: no $c"; return 0; }; done
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d $out/$name -o $name --output-format csv -- $BENCH > $out/$name.log 2>&1
  local rc=$?; echo "[$name] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/$name.log; exit $rc; fi
}
pass sq1 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
pass sq2 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC
pass sq3 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_RD SQ_IFETCH
find $out -name "*counter_collection*.csv" | head
