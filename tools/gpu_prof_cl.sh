#!/bin/bash
# rocprofv3 kernel statistics and counters of the GPU-preset render on the matrix-core
# filter (complex_light_room 1024^2 x 64 spp; k_render<1,0,1,steal,MF>).
# Usage: bash tools/gpu_prof_cl.sh <tag>
tag=${1:-r2p}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/prof_cl_$tag
mkdir -p $out
B="python3 bench.py --workload complex_light --width 1024 --height 1024 --spp 64 --steps 3 --warmup 1 --cpu-seconds 0 --no-parity"
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -1 "$out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then tail -5 "$out/$name.log"; echo "[$name] fatal rc=$rc, stopping"; exit $rc; fi
}
step kt 200 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- $B
step sq1 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d $out/sq1 -o sq1 --output-format csv -- $B
step fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/fetch -o fetch --output-format csv -- $B
