# config 5's bench workload at spp_split 32: its rank-tile test, profile and bench line
bash tools/gpu.sh r3ah \
 "tests:tests/test_gpu_parity.py::test_config5_rank_tile_sets_assemble_to_single_gpu_frame" \
 pmc:complex_light wbench:complex_light
