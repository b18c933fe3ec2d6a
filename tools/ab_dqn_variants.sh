set -o pipefail
mkdir -p gpurun_out/r5i
for r in 1 2; do for v in dq_base dq_mt5db dq_mt5 dq_r40db; do
  RTMI_LIB=reinforcement-light-rays-pathtracer_amd/build/variants/$v/librtmi.so timeout -k 10 120 python3 tools/bench_dqn.py --width 512 --spp 16 --steps 3 > gpurun_out/r5i/${v}_$r.log 2>&1 || exit 1
  echo "$v $r $(tail -1 gpurun_out/r5i/${v}_$r.log | cut -c1-400)"
done; done
