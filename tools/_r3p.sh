# DQN sampler with four cells per Philox draw: tests (unfused default and fused), A/B, kernel stats
V=reinforcement-light-rays-pathtracer_amd/build/variants
bash tools/gpu.sh r3p "tests:tests/test_dqn.py tests/test_neuralq.py" \
 "run:tests_fused:400:RTMI_LIB=$V/dqnfused/librtmi.so python3 -u -m pytest tests/test_dqn.py tests/test_neuralq.py -m gpu -x -q --timeout 240 --timeout-method thread" \
 "run:dqn:300:python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 2" \
 "run:dqn_fused:300:RTMI_LIB=$V/dqnfused/librtmi.so python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 2" \
 "run:kt_unf:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r3p/kt_unf -o kt --output-format csv -- python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 2" \
 "run:kt_fused:300:RTMI_LIB=$V/dqnfused/librtmi.so rocprofv3 --kernel-trace --stats -d gpurun_out/r3p/kt_fused -o kt --output-format csv -- python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 2"
