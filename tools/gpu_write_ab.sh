#!/bin/bash
# WRITE_SIZE of the bench kernel + the render parity tests of the CPU preset
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_cull.py > gpurun_out/wab_tests.log 2>&1 || { tail -30 gpurun_out/wab_tests.log; exit 1; }
tail -1 gpurun_out/wab_tests.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/wab -o wab --output-format csv -- python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-parity > gpurun_out/wab.log 2>&1 || exit 1
python3 - <<'PY'
import csv,glob
f=glob.glob("gpurun_out/wab/**/*counter_collection.csv",recursive=True)[0]
v=[float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "k_render_ps" in r["Kernel_Name"]]
print("WRITE_SIZE KiB per dispatch", sum(v)/len(v), len(v))
PY
timeout -k 10 200 python -u bench.py --cpu-seconds 0 > gpurun_out/wab_bench.log 2>&1 && tail -1 gpurun_out/wab_bench.log | cut -c1-300
