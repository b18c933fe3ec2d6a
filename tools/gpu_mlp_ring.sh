#!/bin/bash
# k_dqn_mlp weight-fragment ring depth A/B (RT_MLP_RING_VGPRS variants from
# tools/build_variants.sh; base = the library before the change): forward pass on 1 M
# archway rays (same Q bit for bit: q_mean printed), interleaved rounds, then the
# archway render at 4 spp for each variant.  Then the BVH-vs-scan bench and a bench line.
# Usage: bash tools/gpu_mlp_ring.sh <tag> variant...
tag=$1; shift
mkdir -p gpurun_out/$tag
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$tag/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(tail -1 gpurun_out/$tag/$name.log | cut -c1-600)"
  if [ $rc -ne 0 ]; then tail -8 "gpurun_out/$tag/$name.log"; echo "[$name] fatal rc=$rc, stopping"; exit $rc; fi
}
V=reinforcement-light-rays-pathtracer_amd/build/variants
for r in 1 2; do
  for v in "$@"; do
    RTMI_LIB=$V/$v/librtmi.so run fwd_${v}_$r 120 python -u tools/bench_dqn.py --no-render --steps 5
  done
done
for v in "$@"; do
  RTMI_LIB=$V/$v/librtmi.so run render_$v 200 python -u tools/bench_dqn.py --spp 4 --steps 2
done
run bench_bvh 240 python -u tools/bench_bvh.py
run bench 300 python -u bench.py --steps 10 --warmup 2
