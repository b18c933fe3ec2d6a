// orc_sort.cpp — TEST INFRASTRUCTURE ONLY (part of oracle/, see rt_oracle.c).
// RadianceTree::sort_radiance_volumes_on_dimension (GPU/radiance_volumes/
// radiance_tree.cu:92-110) sorts with std::sort and the comparator
// position[dim] <; std::sort is not stable, so the tie order of volumes that
// share a coordinate (all volumes of an axis-aligned wall) is the library's.
// This calls the same libstdc++ std::sort so the oracle's tree is the tree
// the reference's algorithm builds.
#include <stdint.h>

#include <algorithm>

extern "C" __attribute__((visibility("default"))) void orc_kd_sort(int32_t* v, int n, const float* pos4, int dim) {
    std::sort(v, v + n, [&](int32_t l, int32_t r) { return pos4[4 * l + dim] < pos4[4 * r + dim]; });
}
