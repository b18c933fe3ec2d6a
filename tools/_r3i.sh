# A/B of the MF filter options on the reverted k_render_ps (per-slot / per-group / 1/2 sign
# thresholds; t values through cross-lane reads or an LDS array), against 615b5df / 193aeaf
L="build/variants/c_615b5df build/variants/c_193aeaf build build/variants/rho1 build/variants/rho2 build/variants/tvlds build/variants/tvrho1"
bash tools/gpu.sh r3i \
 "run:ab_cornell:300:python3 -u tools/ab_render.py $L --split 64 --rounds 7" \
 "run:ab_cl:400:python3 -u tools/ab_render.py $L --split 8 --rounds 2 --scene complex_light_room --preset 1" \
 "run:ab_cg:300:python3 -u tools/ab_render.py $L --split 8 --rounds 3 --preset 1"
