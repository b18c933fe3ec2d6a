#!/bin/bash
# Build librtmi.so variants for in-process A/B timing (tools/ab_render.py).
#   bash tools/build_variants.sh name1 "kflags1" name2 "kflags2" ...
set -e
cd "$(dirname "$0")/../reinforcement-light-rays-pathtracer_amd"
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  make -s BUILD=build/variants/$name KFLAGS="$flags" build/variants/$name/librtmi.so
  make -s BUILD=build/variants/$name KFLAGS="$flags" asm >/dev/null 2>&1 || true
  v=$(grep -A40 "\.name:.*k_renderILi0ELi0ELi0E" build/variants/$name/rt_kernels.s | grep -m1 "\.vgpr_count" | awk '{print $2}')
  echo "$name: $flags vgpr=$v"
done
