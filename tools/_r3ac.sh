# Expected SARSA on the persistent queue with its casts on the matrix-core filter (RT_MF_SARSA)
V=reinforcement-light-rays-pathtracer_amd/build/variants
bash tools/gpu.sh r3ac \
 "run:sarsa:200:python3 tools/bench_sarsa.py --frames 3" \
 "run:sarsa_mf:200:RTMI_LIB=$V/smf/librtmi.so python3 tools/bench_sarsa.py --frames 3" \
 "run:tests_smf:600:RTMI_LIB=$V/smf/librtmi.so python3 -u -m pytest tests/test_sarsa.py -m gpu -x -q --timeout 240 --timeout-method thread"
# per-config measurements of the final build (config 5: every rank's tile set of P = 8 alone)
bash tools/gpu.sh r3ac "run:configs:600:python3 tools/bench_configs.py --only c1 c2 c3 c4 c5 --cpu --out gpurun_out/r3ac/configs.json"
