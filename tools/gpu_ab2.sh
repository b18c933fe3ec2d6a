#!/bin/bash
# GPU tests of the current build, then in-process A/B of render variants.
# Usage: bash tools/gpu_ab2.sh <tag> <pytest-args...> -- <variant ...>
tag=$1; shift
mkdir -p gpurun_out
T=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do T+=("$1"); shift; done; shift
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-3000
  if [ $rc -ne 0 ]; then tail -30 "gpurun_out/$name.log"; echo "[$name] fatal rc=$rc, stopping"; exit $rc; fi
}
run ${tag}_pytest 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread "${T[@]}"
V=""; for v in "$@"; do V="$V build/variants/$v"; done
run ${tag}_ab64 300 python -u tools/ab_render.py $V --rounds 7 --split 64
run ${tag}_ab8 300 python -u tools/ab_render.py $V --rounds 3 --split 8
