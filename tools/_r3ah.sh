# config 5's bench workload at spp_split 32 (its rank-tile test, profile and bench line) and the
# in-frame SARSA TD mode (its test, the whole SARSA suite, the SARSA profile and bench line of
# the rebuilt rt_sarsa.o)
bash tools/gpu.sh r3ah \
 "tests:tests/test_sarsa.py::test_gpu_in_frame_td_mode" \
 "tests:tests/test_gpu_parity.py::test_config5_rank_tile_sets_assemble_to_single_gpu_frame" \
 pmc:door_room_sarsa wbench:door_room_sarsa pmc:complex_light wbench:complex_light tests smoke
