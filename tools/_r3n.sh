# SARSA: the grid's undecided queries walked by the whole wave (RT_SARSA_COOP_KD) -- tests, A/B
# vs HEAD~ and the per-lane walk; DQN: fused sampler with parallel block walks -- tests, A/B
V=reinforcement-light-rays-pathtracer_amd/build/variants
bash tools/gpu.sh r3n "tests:tests/test_sarsa.py tests/test_sarsa_dist.py tests/test_dqn.py" \
 "run:tests_fused:400:RTMI_LIB=$V/dqnfused/librtmi.so python3 -u -m pytest tests/test_dqn.py tests/test_neuralq.py -m gpu -x -q --timeout 240 --timeout-method thread" \
 "run:sarsa_head:200:RTMI_LIB=$V/c_head/librtmi.so python3 tools/bench_sarsa.py --frames 3" \
 "run:sarsa:200:python3 tools/bench_sarsa.py --frames 3" \
 "run:sarsa_nocoop:200:RTMI_LIB=$V/nocoop/librtmi.so python3 tools/bench_sarsa.py --frames 3" \
 "run:dqn:300:python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 2" \
 "run:dqn_fused:300:RTMI_LIB=$V/dqnfused/librtmi.so python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 2"
