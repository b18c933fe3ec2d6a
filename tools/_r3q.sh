# DQN: bounce casts on the matrix-core filter, with and without the fused sampler; the exact
# phase with each lane testing its first candidate itself (RT_MF_FIRST_OWN); SARSA with the
# volume frame, irradiance and qmax in one 64-B record
V=reinforcement-light-rays-pathtracer_amd/build/variants
bash tools/gpu.sh r3q \
 "run:dqn:300:python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 2" \
 "run:dqn_mf:300:RTMI_LIB=$V/dqnmf/librtmi.so python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 2" \
 "run:dqn_fused:300:RTMI_LIB=$V/dqnfused/librtmi.so python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 2" \
 "run:dqn_fmf:300:RTMI_LIB=$V/dqnfmf/librtmi.so python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 2" \
 "run:tests_fmf:400:RTMI_LIB=$V/dqnfmf/librtmi.so python3 -u -m pytest tests/test_dqn.py -m gpu -x -q --timeout 240 --timeout-method thread"
bash tools/gpu.sh r3q \
 "run:ab_cornell:300:python3 -u tools/ab_render.py build build/variants/own1 --split 64 --rounds 9" \
 "run:ab_cl:300:python3 -u tools/ab_render.py build build/variants/own1 --split 8 --rounds 3 --scene complex_light_room --preset 1" \
 "run:ab_cg:300:python3 -u tools/ab_render.py build build/variants/own1 --split 8 --rounds 5 --preset 1"
bash tools/gpu.sh r3q "tests:tests/test_sarsa.py tests/test_sarsa_dist.py" \
 "run:sarsa_head:200:RTMI_LIB=$V/c_head/librtmi.so python3 tools/bench_sarsa.py --frames 3" \
 "run:sarsa_rec:200:python3 tools/bench_sarsa.py --frames 3"
bash tools/gpu.sh r3q \
 "run:accel_cl:300:python3 tools/accel_ab.py --scene complex_light_room --preset 1 --size 512 --spp 64 --split 8" \
 "run:accel_door:300:python3 tools/accel_ab.py --scene door_room --preset 1 --size 512 --spp 64 --split 8"
