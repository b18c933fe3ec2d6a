#!/bin/bash
# In-process A/B of librtmi.so variants on several scenes/presets (images must be
# bit-identical across variants).  Usage: bash tools/gpu_ab_scenes.sh v1 v2 ...
mkdir -p gpurun_out
V=""; for v in "$@"; do V="$V build/variants/$v"; done
for cfg in "cornell 0" "cornell 1" "door_room 1" "archway 1"; do
  set -- $cfg
  timeout -k 10 200 python tools/ab_render.py $V --rounds 3 --split 32 --scene $1 --preset $2 > gpurun_out/ab_$1_$2.log 2>&1 || exit $?
  echo "$1 p$2: $(tail -1 gpurun_out/ab_$1_$2.log)"
done
