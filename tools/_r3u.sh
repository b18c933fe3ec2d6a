# GPU preset on a persistent grid over a (pixel, chunk) queue (k_render_pq): the whole GPU suite,
# then A/B against the per-pixel kernels (RT_RENDER_PQ=0)
bash tools/gpu.sh r3u tests \
 "run:ab_cl:400:python3 -u tools/ab_render.py build build/variants/nopq --split 8 --rounds 3 --scene complex_light_room --preset 1" \
 "run:ab_door:300:python3 -u tools/ab_render.py build build/variants/nopq --split 8 --rounds 3 --scene door_room --preset 1" \
 "run:ab_arch:300:python3 -u tools/ab_render.py build build/variants/nopq --split 8 --rounds 3 --scene archway --preset 1" \
 "run:wbench_cl:400:python3 bench.py --workload complex_light --spp 64 --steps 2 --warmup 1 --cpu-seconds 0 --no-parity"
