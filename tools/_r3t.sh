# GPU-preset sample stealing over the whole wave's pool (RT_STEAL_WAVE): parity tests on that
# build, A/B on complex_light_room, Cornell (GPU preset) and door_room
V=reinforcement-light-rays-pathtracer_amd/build/variants
bash tools/gpu.sh r3t \
 "run:tests_swave:600:RTMI_LIB=$V/swave/librtmi.so python3 -u -m pytest tests/test_gpu_parity.py tests/test_bvh.py tests/test_mf_filter.py -m gpu -x -q --timeout 240 --timeout-method thread" \
 "run:ab_cl:400:python3 -u tools/ab_render.py build build/variants/swave --split 8 --rounds 3 --scene complex_light_room --preset 1" \
 "run:ab_cg:300:python3 -u tools/ab_render.py build build/variants/swave --split 8 --rounds 5 --preset 1" \
 "run:ab_door:300:python3 -u tools/ab_render.py build build/variants/swave --split 8 --rounds 3 --scene door_room --preset 1" \
 "run:ab_cl16:400:python3 -u tools/ab_render.py build build/variants/swave --split 16 --rounds 3 --scene complex_light_room --preset 1"
