#!/bin/bash
# One parametrised GPU-box runner for every measurement of this repo (replaces the
# round-2 single-use tools/gpu_*.sh wrappers).  Each step runs under its own time limit;
# the first failing step ends the call (no GPU work after a fault, abort or timeout).
#
#   bash tools/gpu.sh <tag> <step> [<step> ...]
#
# steps (one shell word each; quote a step that takes arguments):
#   smoke                    __graft_entry__.smoke()
#   tests[:<pytest args>]    pytest -m gpu (default: the whole GPU suite)
#   bench[:<bench args>]     python bench.py --steps 20 --warmup 3 <args>
#   wbench:<workload>        the bench line of a workload with the profiled command's arguments
#                            (so its roofline takes that profile's frames)
#   kt:<workload>            counter-free rocprofv3 --kernel-trace --stats of the bench
#                            workload (profiles/<tag>_<workload>_kernel_stats.csv)
#   pmc:<workload>           PMC passes of the bench workload, summarised into
#                            profiles/<tag>_<workload>_bench_pmc.json (bench.py's roofline)
#   ab:<variant,variant,..>  tools/ab_render.py over build/variants/<v> (same image check)
#   run:<name>:<limit>:<cmd> any command, output in gpurun_out/<tag>/<name>.log
#   configs[:<w1,w2,..>]     for each profile workload (tools/bench_pmc_summary.py WORKLOADS; default:
#                            the five BASELINE configs at their stated sizes): pmc, kt, wbench
# A/B recipes: build the variants here (tools/build_variants.sh name "flags" ...), then
#   ab:<v1,v2>                         Cornell frame, same image checked (tools/ab_render.py)
#   run:x:600:'RTMI_LIB=.../variants/<v>/librtmi.so python3 tools/bench_sarsa.py' (or bench_dqn.py)
# Outputs: gpurun_out/<tag>/ (gpurun copies only gpurun_out/ back); the summaries meant for
# profiles/ go to gpurun_out/<tag>/profiles/.  Here, without a GPU:
#   bash tools/gpu.sh <tag> collect      copies them into profiles/
set -o pipefail
tag=$1; shift
cd "$(dirname "$0")/.." || exit 1
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp

run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(tail -1 "$out/$name.log" | cut -c1-1500)"
  if [ $rc -ne 0 ]; then tail -25 "$out/$name.log"; echo "[$name] fatal rc=$rc, stopping"; exit $rc; fi
}

bench_cmd() {  # workload [steps] -> the bench command the profiles are taken of (one source:
               # tools/bench_pmc_summary.py WORKLOADS); kt runs it with more steps
  local a
  a=$(python3 tools/bench_pmc_summary.py --args "$1") || exit 2
  [ -n "$2" ] && a=$(echo "$a" | sed "s/--steps [0-9]*/--steps $2/")
  echo "python3 bench.py $a"
}

pmc_pass() {  # workload name counters...
  local w=$1 name=$2; shift 2
  local d=$out/pmc_$w
  mkdir -p "$d"
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace -d "$d/$name" -o "$name" --output-format csv \
      -- $(bench_cmd "$w") > "$d/$name.log" 2>&1
  local rc=$?
  echo "[pmc $w $name] rc=$rc"
  if [ $rc -ne 0 ]; then tail -8 "$d/$name.log"; echo "[pmc $w $name] fatal rc=$rc, stopping"; exit $rc; fi
}

for step in "$@"; do
  kind=${step%%:*}; arg=""
  [ "$kind" != "$step" ] && arg=${step#*:}
  case $kind in
    smoke) run smoke 240 python3 -u -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run "tests" 900 python3 -u -m pytest ${arg:-tests} -m gpu -x -q --timeout 240 --timeout-method thread ;;
    bench) run "bench${arg:+_$(echo "$arg" | tr -c 'a-z0-9' '_')}" 400 python3 -u bench.py --steps 20 --warmup 3 $arg ;;
    wbench)
      run "wbench_$arg" 400 $(bench_cmd "$arg" | sed 's/--cpu-seconds 0//') ;;
    kt)
      w=${arg:-cornell}
      steps=""; [ "$w" = cornell ] && steps=40  # (others: the profiled command's own frames)
      run "kt_$w" 400 rocprofv3 --kernel-trace --stats -d "$out/kt_$w" -o kt --output-format csv -- $(bench_cmd "$w" $steps)
      mkdir -p "$out/profiles"
      cp "$out/kt_$w/kt_kernel_stats.csv" "$out/profiles/${tag}_${w}_kernel_stats.csv"
      rm -rf "$out/kt_$w" ;;  # (the traces of a 10k-launch frame exceed what gpurun copies back)
    pmc)
      w=${arg:-cornell}
      pmc_pass "$w" fetch FETCH_SIZE
      pmc_pass "$w" write WRITE_SIZE
      pmc_pass "$w" sq1 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU
      pmc_pass "$w" sq2 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_BRANCH
      pmc_pass "$w" sq3 SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_F32 GRBM_GUI_ACTIVE
      run "pmc_summary_$w" 60 python3 tools/bench_pmc_summary.py "$out/pmc_$w" "$tag" "$w" "$out/profiles"
      # (the box's scratch tree: later bench / wbench steps of this call find the profile)
      cp "$out"/profiles/*_bench_pmc.json profiles/
      rm -rf "$out/pmc_$w" ;;  # raw counter CSVs: summarised above
    collect)
      mkdir -p profiles
      for f in "$out"/profiles/*; do [ -e "$f" ] && cp -v "$f" profiles/; done
      for f in "$out"/smoke.log "$out"/tests.log "$out"/bench*.log "$out"/wbench*.log; do [ -e "$f" ] && cp "$f" "profiles/${tag}_$(basename "$f")"; done ;;
    configs)
      for w in $(echo "${arg:-cornell_c1,cornell,door_room_sarsa,archway_dqn,complex_light}" | tr ',' ' '); do
        "$0" "$tag" "pmc:$w" "kt:$w" "wbench:$w" || exit $?
      done ;;
    ab) run "ab" 400 python3 -u tools/ab_render.py $(echo "$arg" | tr ',' '\n' | sed 's#^#build/variants/#') --split 64 --rounds 7 ;;
    run)
      name=${arg%%:*}; rest=${arg#*:}; lim=${rest%%:*}; cmd=${rest#*:}
      run "$name" "$lim" bash -c "$cmd" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu.sh $tag] done"
