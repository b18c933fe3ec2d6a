bash tools/gpu.sh r3c tests \
 "run:ab_cornell:300:python3 -u tools/ab_render.py build/variants/r3a build/variants/pp0 build build/variants/cap128 build/variants/w5 --split 64 --rounds 9" \
 "run:ab_cl:300:python3 -u tools/ab_render.py build/variants/r3a build/variants/pp0 build --split 8 --rounds 3 --scene complex_light_room --preset 1" \
 "run:ab_cg:300:python3 -u tools/ab_render.py build/variants/r3a build/variants/camoff build --split 8 --rounds 5 --preset 1" \
 "run:cand_old:200:RTMI_LIB=reinforcement-light-rays-pathtracer_amd/build/variants/r3a/librtmi.so python3 tools/bench_mf_filter.py --scene complex_light_room --reps 1" \
 "run:cand_new:200:python3 tools/bench_mf_filter.py --scene complex_light_room --reps 1" \
 "run:cand_new_c:200:python3 tools/bench_mf_filter.py --reps 1" \
 "run:sarsa_base:200:python3 tools/bench_sarsa.py --frames 3" \
 "run:sarsa_mf:200:python3 tools/bench_sarsa.py --frames 3 --lib build/variants/sarsamf"
