# occupancy A/B of k_render_ps: pair cap 128 (LDS 32.5 KB per workgroup: 5 per CU) with 4 / 5 / 6 waves per SIMD
L="build build/variants/c128 build/variants/w5c128 build/variants/w6c128"
bash tools/gpu.sh r3l "run:ab_cornell:300:python3 -u tools/ab_render.py $L --split 64 --rounds 9"
