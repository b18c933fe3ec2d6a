#!/bin/bash
# SQ counter passes over the default bench workload for the matrix-core filter work
# (kernel trace + three SQ passes), raw CSVs under gpurun_out/pmc_<tag>.
tag=${1:-mf}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/pmc_$tag
mkdir -p $out
BENCH="python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-parity"
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$out/$name.log"; echo "[$name] fatal rc=$rc, stopping"; exit $rc; fi
}
step kt 240 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- $BENCH
step sq1 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace -d $out/sq1 -o sq1 --output-format csv -- $BENCH
step sq2 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_BRANCH --kernel-trace -d $out/sq2 -o sq2 --output-format csv -- $BENCH
step sq3 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d $out/sq3 -o sq3 --output-format csv -- $BENCH
