#!/bin/bash
# A/B: the GPU-preset Cornell render on the matrix-core filter with the camera outside
# the image bound (camout) vs the fp32 filter (base); parity of the render cases on camout.
tag=${1:-r2q}
mkdir -p gpurun_out/$tag
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$tag/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(tail -1 gpurun_out/$tag/$name.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then tail -20 "gpurun_out/$tag/$name.log"; echo "[$name] fatal rc=$rc, stopping"; exit $rc; fi
}
V=reinforcement-light-rays-pathtracer_amd/build/variants
RTMI_LIB=$V/camout/librtmi.so run parity 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "render_matches_oracle or tile_render or cornell_matches"
for r in 1 2; do
  for v in base camout; do
    RTMI_LIB=$V/$v/librtmi.so run ab_${v}_$r 120 python -u tools/ab_cornell_gpu.py
  done
done
