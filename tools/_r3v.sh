# Expected SARSA on the persistent (pixel, chunk) queue (k_sarsa_render_pq): the whole GPU
# suite, then frames against the per-pixel kernel (RT_SARSA_PQ=0)
V=reinforcement-light-rays-pathtracer_amd/build/variants
bash tools/gpu.sh r3v tests \
 "run:sarsa_nopq:200:RTMI_LIB=$V/nopq/librtmi.so python3 tools/bench_sarsa.py --frames 3" \
 "run:sarsa_pq:200:python3 tools/bench_sarsa.py --frames 3" \
 "run:sarsa_cl_nopq:300:RTMI_LIB=$V/nopq/librtmi.so python3 tools/bench_sarsa.py --scene complex_light_room --frames 2" \
 "run:sarsa_cl_pq:300:python3 tools/bench_sarsa.py --scene complex_light_room --frames 2"
