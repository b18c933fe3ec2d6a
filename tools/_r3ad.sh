# the persistent GPU-preset kernel held to 5 / 6 waves per SIMD (RT_MF_RENDER_WAVES)
bash tools/gpu.sh r3ad \
 "run:ab_cl:400:python3 -u tools/ab_render.py build build/variants/w5 build/variants/w6 --split 8 --rounds 3 --scene complex_light_room --preset 1" \
 "run:ab_door:300:python3 -u tools/ab_render.py build build/variants/w5 build/variants/w6 --split 8 --rounds 3 --scene door_room --preset 1"
