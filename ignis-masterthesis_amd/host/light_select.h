// Tables of the non-uniform NEE light selectors (host side, built at upload).
//
// The reference picks the selector when it generates the technique's code
// (LoaderLight::generateLightSelector, LoaderLight.cpp:423-453):
//   "simple":    a CDF over the finite lights' flux (generateLightSelectionCDF,
//                LoaderLight.cpp:455-476; CDF::computeForArray, CDF.cpp:11-40),
//                sampled by make_cdf_light_selector (light/light_selector.art:46-75);
//   "hierarchy": a light BVH (LightHierarchy::setup, LightHierarchy.cpp:75-118,
//                over PointBvh, container/PointBvh.inl) walked by
//                light/light_hierarchy.art (Moreau and Clarberg 2019);
// anything else, one light or none: the uniform selector.
#pragma once

#include "igx_scene.h"

#include <cstdint>
#include <vector>

namespace igx {

struct LightSelectTables {
    int selector = IGX_SELECT_UNIFORM; // the selector in effect
    std::vector<float> cdf;            // simple: [c_1, ..., c_{n-1}, 1] (the leading 0 is implicit)
    // hierarchy: per finite light the left/right code (bit d = 1: right at depth d),
    // padded to a multiple of 4, then 8 floats per tree entry:
    // position.xyz, flux (negative: no direction), direction.xyz, index
    // (bit pattern of an int: >= 0 light id of a leaf, -(left child + 1) of an inner entry)
    std::vector<uint32_t> hierarchy;
};

// `finite` = the finite lights in selector order (light ids 0..n-1);
// `light_count` = finite + infinite lights.
LightSelectTables build_light_select(int selector, int light_count, const std::vector<igx_light>& finite);

} // namespace igx
