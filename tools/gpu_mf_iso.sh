#!/bin/bash
# hit test alone: fp32 filter vs matrix-core filter kernels (rocprofv3 kernel stats)
tag=${1:-iso}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- python3 tools/bench_mf_filter.py > $out/run.log 2>&1 || { tail -5 $out/run.log; exit 1; }
tail -1 $out/run.log
python3 -c "
import csv
for r in csv.DictReader(open('$out/kt/kt_kernel_stats.csv')):
    if 'intersect' in r['Name']: print(r['Name'][:60], r['Calls'], r['AverageNs'])"
