#!/bin/bash
# rocprofv3 passes over the default bench workload (one run each): kernel trace +
# stats, FETCH_SIZE, WRITE_SIZE, and two SQ passes.  Then summarise into
# profiles/<tag>_bench_pmc.json (tools/bench_pmc_summary.py), the file bench.py reads.
# Usage: bash tools/gpu_bench_pmc.sh <tag>
tag=${1:-r2}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/pmc_$tag
mkdir -p $out
BENCH="python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-parity"
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$out/$name.log"; echo "[$name] fatal rc=$rc, stopping"; exit $rc; fi
}
step kt 240 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- $BENCH
step fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/fetch -o fetch --output-format csv -- $BENCH
step write 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $out/write -o write --output-format csv -- $BENCH
step sq1 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace -d $out/sq1 -o sq1 --output-format csv -- $BENCH
step sq2 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_BRANCH --kernel-trace -d $out/sq2 -o sq2 --output-format csv -- $BENCH
# matrix-core counters (k_render_ps casts its bounce rays on the MFMA filter); not fatal
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_BF16 GRBM_GUI_ACTIVE --kernel-trace -d $out/sq3 -o sq3 --output-format csv -- $BENCH > $out/sq3.log 2>&1; echo "[sq3] rc=$?"
python3 tools/bench_pmc_summary.py $out $tag
