# k_render_ps: each lane tests its first 1 / 2 / 3 candidates itself before the shared phase
V=reinforcement-light-rays-pathtracer_amd/build/variants
bash tools/gpu.sh r3aa \
 "run:ab_cornell:300:python3 -u tools/ab_render.py build build/variants/own2 build/variants/own3 --split 64 --rounds 9" \
 "run:tests_own2:600:RTMI_LIB=$V/own2/librtmi.so python3 -u -m pytest tests/test_gpu_parity.py tests/test_mf_filter.py -m gpu -x -q --timeout 240 --timeout-method thread"
