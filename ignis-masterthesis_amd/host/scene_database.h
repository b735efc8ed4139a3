// The reference's scene tables (src/runtime/table/{DynTable,FixTable,
// SceneDatabase}.h) with the same members and padding rules, so the IG::Device
// facade (Device.h) takes the same SceneSettings as the reference's device,
// and igx's own loader can emit them (serialize_scene) the way the reference
// loader does (LoaderEntity.cpp:32-205, TriMeshProvider.cpp:480-617,
// SphereProvider.cpp:10-53).
#pragma once

#include "igx_scene.h"

#include <cstddef>
#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

namespace IG {

using uint8 = uint8_t;
using uint32 = uint32_t;
using uint64 = uint64_t;

struct LookupEntry { // table/DynTable.h:6-10
    uint32 TypeID;
    uint32 Flags;
    uint64 Offset;
};
static_assert(sizeof(LookupEntry) == sizeof(igx_lookup_entry), "DynTable lookup layout");

class DynTable { // table/DynTable.h:12-34
public:
    size_t entryCount() const { return mLookups.size(); }
    void reserve(size_t size) { mData.reserve(size); }
    // pads by a full `alignment` even when the data is already aligned (DynTable.h:20-23)
    std::vector<uint8>& addLookup(uint32 typeID, uint32 flags, size_t alignment) {
        if (alignment != 0 && !mData.empty()) mData.resize(mData.size() + alignment - mData.size() % alignment);
        mLookups.push_back(LookupEntry{typeID, flags, (uint64)mData.size()});
        return mData;
    }
    const std::vector<LookupEntry>& lookups() const { return mLookups; }
    const std::vector<uint8>& data() const { return mData; }
    size_t currentOffset() const { return mData.size(); }

private:
    std::vector<LookupEntry> mLookups;
    std::vector<uint8> mData;
};

class FixTable { // table/FixTable.h:10-30
public:
    void reserve(size_t size) { mData.reserve(size); }
    std::vector<uint8>& addEntry(size_t alignment) {
        if (alignment != 0 && !mData.empty()) mData.resize(mData.size() + alignment - mData.size() % alignment);
        mCount++;
        return mData;
    }
    const std::vector<uint8>& data() const { return mData; }
    size_t currentOffset() const { return mData.size(); }
    size_t entryCount() const { return mCount; }

private:
    size_t mCount = 0;
    std::vector<uint8> mData;
};

struct SceneBVH { // table/SceneDatabase.h:8-11
    std::vector<uint8> Nodes;
    std::vector<uint8> Leaves;
};

struct BoundingBox {
    float min[3] = {0, 0, 0};
    float max[3] = {0, 0, 0};
};

struct SceneDatabase { // table/SceneDatabase.h:13-20
    std::unordered_map<std::string, SceneBVH> SceneBVHs;
    std::unordered_map<std::string, DynTable> DynTables;
    std::unordered_map<std::string, FixTable> FixTables;
    float SceneRadius = 0;
    BoundingBox SceneBBox;
    size_t MaterialCount = 0;
};

// ShapeProvider::id() (TriMeshProvider.h:13, SphereProvider.h:12) and the
// SceneBVHs keys (ShapeProvider::identifier(), LoaderEntity.cpp:190)
constexpr uint32 kTrimeshProviderID = 0;
constexpr uint32 kSphereProviderID = 1;

// igx_database_view over a SceneDatabase (valid while the database lives)
struct DatabaseViewStorage {
    igx_database_view view{};
    std::vector<igx_db_table> leaves;

    explicit DatabaseViewStorage(const SceneDatabase& db) {
        auto fix = [&](const char* name) {
            igx_db_table t{};
            auto it = db.FixTables.find(name);
            if (it != db.FixTables.end()) {
                t.data = it->second.data().data();
                t.bytes = it->second.data().size();
                t.count = it->second.entryCount();
            }
            return t;
        };
        view.entities = fix("entities");
        view.trimesh_primbvh = fix("trimesh_primbvh");
        if (auto it = db.DynTables.find("shapes"); it != db.DynTables.end()) {
            view.shapes.data = it->second.data().data();
            view.shapes.bytes = it->second.data().size();
            view.shapes.lookups = reinterpret_cast<const igx_lookup_entry*>(it->second.lookups().data());
            view.shapes.count = it->second.entryCount();
        }
        view.trimesh_type_id = kTrimeshProviderID;
        view.sphere_type_id = kSphereProviderID;
        for (const auto& kv : db.SceneBVHs) {
            igx_db_table t{};
            t.data = kv.second.Leaves.data();
            t.bytes = kv.second.Leaves.size();
            leaves.push_back(t);
        }
        view.scene_bvh_leaves = leaves.data();
        view.num_scene_bvhs = (uint32_t)leaves.size();
        for (int i = 0; i < 3; ++i) {
            view.scene_bbox_min[i] = db.SceneBBox.min[i];
            view.scene_bbox_max[i] = db.SceneBBox.max[i];
        }
    }
    DatabaseViewStorage(const DatabaseViewStorage&) = delete;
    DatabaseViewStorage& operator=(const DatabaseViewStorage&) = delete;
};

// Write a loaded scene into the reference's tables, as the reference loader
// does for a GPU target: FixTables["entities"], DynTables["shapes"],
// FixTables["trimesh_primbvh"] (Node2 + Tri1 BLAS of every trimesh shape,
// built by host/bvh_build.cpp in place of madmann91/bvh) and
// SceneBVHs["trimesh" | "sphere"] (Node2 + EntityLeaf1 TLAS per provider).
// `shading` receives the tables the reference turns into shader code; it
// points into `desc`, which must outlive it.
void serialize_scene(const igx_scene_desc& desc, SceneDatabase& db, igx_shading_view& shading);

} // namespace IG
