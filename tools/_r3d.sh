V=reinforcement-light-rays-pathtracer_amd/build/variants
bash tools/gpu.sh r3d tests \
 "run:ab_cornell:300:python3 -u tools/ab_render.py build/variants/r3a build build/variants/w5c build/variants/rhog5 build/variants/rhoc5 --split 64 --rounds 9" \
 "run:ab_cl:300:python3 -u tools/ab_render.py build/variants/r3a build build/variants/w5c build/variants/rhog5 build/variants/rhoc5 --split 8 --rounds 3 --scene complex_light_room --preset 1" \
 "run:cand_c:200:python3 tools/bench_mf_filter.py --reps 1" \
 "run:cand_cl:200:python3 tools/bench_mf_filter.py --scene complex_light_room --reps 1" \
 "run:dqn_unf:300:RTMI_LIB=$V/dqnunf/librtmi.so python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 2" \
 "run:dqn_fused:300:python3 tools/bench_dqn.py --scene archway --width 512 --spp 16 --steps 2"
