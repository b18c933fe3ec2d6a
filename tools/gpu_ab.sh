#!/bin/bash
# in-process A/B of librtmi variants (tools/ab_render.py), Cornell CPU preset bench config
#   bash tools/gpu_ab.sh <tag> variant1 variant2 ...
set -o pipefail
tag=$1; shift
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
args=""
for v in "$@"; do args="$args build/variants/$v"; done
timeout -k 10 300 python3 tools/ab_render.py $args --split 64 --rounds 7 > gpurun_out/${tag}_ab.json 2>gpurun_out/${tag}_ab.err || { tail -5 gpurun_out/${tag}_ab.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/${tag}_ab.json'))
for k,v in d['results'].items(): print(k.split('/')[-1], v['ms_median'], v['gcasts_s'], v['same_image'])"
