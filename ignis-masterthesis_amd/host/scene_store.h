// Owner of the arrays an igx_scene_desc points into (igx_scene handle), shared
// by the JSON loader (scene_loader.cpp) and the SceneDatabase adapter
// (db_adapter.cpp).
#pragma once

#include "igx_scene.h"

#include <cstdint>
#include <string>
#include <vector>

namespace igx {

struct SceneStore {
    igx_scene_desc desc{};
    std::vector<std::vector<float>> vtx, nrm, tex;
    std::vector<std::vector<uint32_t>> idx;
    std::vector<std::vector<uint8_t>> bvh; // reference BLAS blobs (igx_shape::ref_bvh)
    std::vector<igx_mesh> meshes;
    std::vector<igx_shape> shapes;
    std::vector<igx_entity> entities;
    std::vector<igx_material> materials;
    std::vector<igx_light> lights;
    // names (JSON loader only): entity names, and per material id its BSDF
    // name and emissive entity (LoaderContext::Material, LoaderContext.h:19-27)
    std::vector<std::string> entity_names;
    std::vector<std::string> material_bsdf, material_entity;

    // point desc at the arrays (after they stop growing)
    void publish() {
        desc.num_meshes = (uint32_t)meshes.size();
        desc.meshes = meshes.data();
        desc.num_shapes = (uint32_t)shapes.size();
        desc.shapes = shapes.data();
        desc.num_entities = (uint32_t)entities.size();
        desc.entities = entities.data();
        desc.num_materials = (uint32_t)materials.size();
        desc.materials = materials.data();
        desc.num_lights = (uint32_t)lights.size();
        desc.lights = lights.data();
    }
};

} // namespace igx

struct igx_scene {
    igx::SceneStore store;
};
