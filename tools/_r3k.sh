# bench lines of configs 3-5 with the r3j profiles; per-phase cycles of k_render_ps (RT_PROF
# build); SARSA and DQN casts on the matrix-core filter vs the fp32 filter
bash tools/gpu.sh r3k wbench:door_room_sarsa wbench:archway_dqn wbench:complex_light \
 "run:psprof:120:RT_PS_PROF=1 RTMI_LIB=reinforcement-light-rays-pathtracer_amd/build/variants/prof/librtmi.so python3 bench.py --steps 2 --warmup 0 --cpu-seconds 0 --no-parity" \
 "run:sarsa:200:python3 tools/bench_sarsa.py --frames 3" \
 "run:sarsa_mf:200:RTMI_LIB=reinforcement-light-rays-pathtracer_amd/build/variants/sarsamf/librtmi.so python3 tools/bench_sarsa.py --frames 3" \
 "run:dqn:300:python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 2" \
 "run:dqn_mf:300:RTMI_LIB=reinforcement-light-rays-pathtracer_amd/build/variants/dqnmf/librtmi.so python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 2"
