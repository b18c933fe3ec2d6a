# A/B: round-2 kernels (615b5df), 193aeaf, HEAD; DQN fused vs unfused; SARSA frame time
bash tools/gpu.sh r3h \
 "run:ab_cornell:300:python3 -u tools/ab_render.py build/variants/c_615b5df build/variants/c_193aeaf build --split 64 --rounds 9" \
 "run:ab_cl:300:python3 -u tools/ab_render.py build/variants/c_615b5df build/variants/c_193aeaf build --split 8 --rounds 3 --scene complex_light_room --preset 1" \
 "run:ab_cg:300:python3 -u tools/ab_render.py build/variants/c_615b5df build/variants/c_193aeaf build --split 8 --rounds 5 --preset 1" \
 "run:dqn_unf:300:RTMI_LIB=reinforcement-light-rays-pathtracer_amd/build/variants/dqnunf/librtmi.so python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 2" \
 "run:dqn_fused:300:python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 2" \
 "run:sarsa_r2:200:RTMI_LIB=reinforcement-light-rays-pathtracer_amd/build/variants/c_615b5df/librtmi.so python3 tools/bench_sarsa.py --frames 3" \
 "run:sarsa:200:python3 tools/bench_sarsa.py --frames 3"
