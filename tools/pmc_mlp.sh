#!/bin/bash
# PMC passes of the DQN forward alone (tools/bench_dqn.py --no-render: 1 M rays per launch),
# one counter group per rocprofv3 run; CSVs under gpurun_out/<tag>/mlp_pmc/.
tag=${1:-mlp}
out=gpurun_out/$tag/mlp_pmc
mkdir -p "$out"
export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d "$out/$name" -o "$name" --output-format csv \
      -- python3 tools/bench_dqn.py --no-render --steps 5 > "$out/$name.log" 2>&1
  local rc=$?
  echo "[pmc $name] rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$out/$name.log"; exit $rc; }
}
pass a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE
pass b SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU
pass c SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD SQ_WAVES SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_VALU_MFMA_BF16
echo "[pmc_mlp] done"
