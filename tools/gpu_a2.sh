set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/ab_render.py build/variants/ps1 build/variants/rngcheap build/variants/w6 --rounds 5 --split 64 > gpurun_out/a2_ab64.log 2>&1 || exit $?
tail -1 gpurun_out/a2_ab64.log
bash tools/gpu_profile.sh r2a2 || exit $?
bash tools/gpu_pmc.sh r2a2pmc || exit $?
