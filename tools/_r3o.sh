# kernel statistics of the DQN frame, unfused (default) vs fused forward+sampler
V=reinforcement-light-rays-pathtracer_amd/build/variants
bash tools/gpu.sh r3o \
 "run:kt_unf:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r3o/kt_unf -o kt --output-format csv -- python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 2" \
 "run:kt_fused:300:RTMI_LIB=$V/dqnfused/librtmi.so rocprofv3 --kernel-trace --stats -d gpurun_out/r3o/kt_fused -o kt --output-format csv -- python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 2"
