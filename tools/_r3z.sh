# k_render_ps on a persistent grid of waves (RT_PS_PERSIST): parity tests on that build, A/B
V=reinforcement-light-rays-pathtracer_amd/build/variants
bash tools/gpu.sh r3z \
 "run:tests_pspw:600:RTMI_LIB=$V/pspw/librtmi.so python3 -u -m pytest tests/test_gpu_parity.py tests/test_cull.py tests/test_mf_filter.py -m gpu -x -q --timeout 240 --timeout-method thread" \
 "run:ab_cornell:300:python3 -u tools/ab_render.py build build/variants/pspw --split 64 --rounds 9"
