cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/bis
for v in c_615b5df c_193aeaf; do
  RTMI_LIB=reinforcement-light-rays-pathtracer_amd/build/variants/$v/librtmi.so timeout -k 10 300 python3 -u -m pytest tests/test_mf_filter.py tests/test_gpu_parity.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/bis/$v.log 2>&1
  rc=$?; echo "[$v] rc=$rc"; tail -25 gpurun_out/bis/$v.log; [ $rc -le 1 ] || exit $rc
done
