mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_tiles_dist.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_steal.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_steal.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
P=$PWD/reinforcement-light-rays-pathtracer_amd/build/variants
for r in 1 2; do for v in nosteal steal; do
  RTMI_LIB=$P/$v/librtmi.so timeout -k 10 200 python bench.py --cpu-seconds 0 --no-parity --steps 20 > gpurun_out/ab_$v.log 2>&1 || exit $?
  echo "$v: $(tail -1 gpurun_out/ab_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done; done
