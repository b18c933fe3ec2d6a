# config 5's rank tile sets at P = 8 with finer chunks (spp_split 16 / 32): each rank launch's tail
bash tools/gpu.sh r3ag \
 "run:c5_s16:400:python3 tools/bench_configs.py --only c5 --cpu --c5-split 16 --out gpurun_out/r3ag/c5_s16.json" \
 "run:c5_s32:400:python3 tools/bench_configs.py --only c5 --cpu --c5-split 32 --out gpurun_out/r3ag/c5_s32.json" \
 "run:c5_s8:400:python3 tools/bench_configs.py --only c5 --cpu --c5-split 8 --out gpurun_out/r3ag/c5_s8.json"
