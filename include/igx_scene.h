/*
 * igx_scene.h — scene description handed across the drop-in boundary.
 *
 * This is the data the reference's loader hands to its device through
 * `IG::SceneSettings` (src/runtime/device/Device.h:25-30), restated as plain C
 * structs.  The reference passes a `SceneDatabase*` whose tables are produced by
 * `TriMeshProvider::handle` (src/runtime/shape/TriMeshProvider.cpp:480-617),
 * `SphereProvider::handle` (src/runtime/shape/SphereProvider.cpp:10-53),
 * `LoaderEntity::load` (src/runtime/loader/LoaderEntity.cpp:32-205) and the
 * light/BSDF serialisers.  The reference turns materials and lights into JIT
 * code; here they are data (material and light tables), because there is no
 * Artic JIT in this build (SURVEY.md §7 "hard parts").
 *
 * All pointers inside an igx_scene_desc are owned by the igx_scene handle that
 * produced them (igx_scene_load_*); igx_upload_scene copies what it needs.
 */
#ifndef IGX_SCENE_H
#define IGX_SCENE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- shapes ------------------------------------------------------------ */
enum { IGX_SHAPE_TRIMESH = 0, IGX_SHAPE_SPHERE = 1 };

/* Object-space triangle mesh after the shape's own transform and flip_normals
 * were baked in (TriMeshProvider.cpp:529-541).  Indices are 3 per face. */
typedef struct igx_mesh {
    uint32_t num_vertices;
    uint32_t num_faces;
    const float* vertices;   /* 3 * num_vertices */
    const float* normals;    /* 3 * num_vertices (unit) */
    const float* texcoords;  /* 2 * num_vertices */
    const uint32_t* indices; /* 3 * num_faces */
} igx_mesh;

typedef struct igx_shape {
    int32_t type;        /* IGX_SHAPE_* */
    int32_t mesh;        /* index into meshes for TRIMESH, -1 otherwise */
    float sphere[4];     /* origin.xyz, radius for SPHERE */
    float bbox_min[3];   /* local bbox, inflated by 1e-5 (TriMeshProvider.cpp:537-538) */
    float bbox_max[3];
    /* plane representation (TriMesh::getAsPlane, mesh/TriMesh.cpp:520-634) */
    int32_t is_plane;
    float plane_origin[3], plane_x[3], plane_y[3];
    float plane_tex[8];  /* 4 texcoords */
    /* Optional prebuilt BLAS in the reference's GPU layout: one
     * FixTables["trimesh_primbvh"] entry (TriMeshProvider.cpp:307-326, 361-369):
     * u32 node_count, tri_count, 0, 0; Node2[node_count] (64 B,
     * traversal/mapping_gpu.art:3-7; child > 0 inner index + 1, < 0 ~first Tri1,
     * 0 empty); Tri1[tri_count] (48 B, shapes/trimesh.art:107-114; prim_id bit 31
     * ends a leaf).  NULL: igx builds the BLAS itself (host/bvh_build.cpp). */
    const uint8_t* ref_bvh;
    uint64_t ref_bvh_bytes;
} igx_shape;

/* ---- entities ---------------------------------------------------------- */
/* Matrices are 3x4 row-major: m[r*4+c].  normal is 3x3 row-major.  The
 * reference stores the same three matrices per entity, 36 floats
 * (LoaderEntity.cpp:150-162), column-major. */
typedef struct igx_entity {
    int32_t shape;
    int32_t material;
    uint32_t flags;         /* visibility flags 0x1 camera 0x2 light 0x4 bounce 0x8 shadow */
    float to_global[12];
    float to_local[12];
    float normal[9];        /* inverse-transpose of the linear part of to_global */
    float bbox_min[3];      /* world-space bbox = local bbox transformed (LoaderEntity.cpp:141) */
    float bbox_max[3];
} igx_entity;

/* ---- materials --------------------------------------------------------- */
enum {
    IGX_BSDF_DIFFUSE    = 0, /* Lambert / Oren-Nayar (bsdf/diffuse.art) */
    IGX_BSDF_DIELECTRIC = 1, /* pure (smooth) dielectric (bsdf/dielectric.art) */
    IGX_BSDF_CONDUCTOR  = 2, /* mirror / pure / rough conductor (bsdf/conductor.art) */
    IGX_BSDF_PLASTIC    = 3, /* Fresnel mix of diffuse and a conductor lobe (bsdf/plastic.art) */
    IGX_BSDF_PRINCIPLED = 4  /* Disney BSDF (bsdf/principled.art) */
};
/* microfacet distribution of conductor / plastic lobes (BSDF::setupRoughness, BSDF.cpp:53-99) */
enum { IGX_MICROFACET_DELTA = 0, IGX_MICROFACET_VNDF_GGX = 1, IGX_MICROFACET_GGX = 2, IGX_MICROFACET_BECKMANN = 3 };

typedef struct igx_material {
    int32_t bsdf_type;     /* IGX_BSDF_* */
    int32_t light;         /* index of the area light emitting from this material, -1 if none */
    int32_t thin;          /* dielectric: thin interface */
    int32_t distribution;  /* IGX_MICROFACET_* (conductor, plastic) */
    float kd[3];           /* diffuse reflectance */
    float ks[3];           /* specular reflectance */
    float kt[3];           /* specular transmittance */
    float ext_ior, int_ior;
    float eta[3];          /* conductor complex ior: real part */
    float kappa[3];        /* conductor complex ior: imaginary part */
    float alpha_u, alpha_v;/* microfacet roughness (compute_explicit, core/microfacet.art:395-402) */
    float diffuse_alpha;   /* Oren-Nayar roughness, 0 = Lambert */
    float pad;
    /* principled (PrincipledBSDF.cpp:11-60): kd = base_color, alpha_u / alpha_v =
     * roughness_u / roughness_v (already through compute_roughness), thin */
    float ior, diffuse_transmission, specular_transmission, specular_tint, flatness, metallic;
    float sheen, sheen_tint, clearcoat, clearcoat_gloss, clearcoat_roughness;
    int32_t clearcoat_top_only;
    /* diffuse reflectance given by a shading expression the loader recognises
     * (ShadingTree / PExpr): IGX_TEXTURE_CHECKER is
     * select(checkerboard(uvw * tex_scale) == 1, tex_kd1, kd), the 3D
     * checkerboard of texture/checkerboard.art:2 on the surface's texture
     * coordinates (u, v, 0) (shapes/trimesh.art:25); IGX_TEXTURE_NONE: kd */
    int32_t texture;
    float tex_scale;
    float tex_kd1[3];
} igx_material;

enum { IGX_TEXTURE_NONE = 0, IGX_TEXTURE_CHECKER = 1 };

/* ---- lights ------------------------------------------------------------ */
enum {
    IGX_LIGHT_PLANE = 1, /* area light on a planar entity: make_plane_area_emitter (light/area.art:107-240) */
    IGX_LIGHT_ENV   = 2, /* constant environment, spherical sampling (light/env.art:73-98) */
    IGX_LIGHT_POINT = 3, /* light/point.art:1-18 */
    IGX_LIGHT_SPOT  = 4, /* light/spot.art:8-60 */
    IGX_LIGHT_DIRECTIONAL = 5, /* light/directional.art:1-19 */
    IGX_LIGHT_SUN   = 6, /* light/sun.art:4-30 (delta, infinite) */
    IGX_LIGHT_SPHERE = 7, /* area light on a (near-)spherical entity: make_sphere_area_emitter (light/area.art:240-293) */
    IGX_LIGHT_MESH  = 8  /* area light on any triangle entity: make_shape_area_emitter (light/area.art:45-105) */
};

typedef struct igx_light {
    int32_t type;
    int32_t entity;        /* area lights: emitting entity, -1 otherwise */
    float radiance[3];     /* radiance (area/env), intensity (point/spot), irradiance (directional/sun) */
    float origin[3];       /* plane origin / point position / spot position / sphere centre (object space) */
    float x_axis[3];       /* plane */
    float y_axis[3];       /* plane */
    float normal[3];       /* plane normal, spot / directional / sun propagation direction */
    float area;            /* plane area; sphere: emitter area, compute_ellipsoid_area (shapes/sphere.art:21-27) */
    float cutoff, falloff; /* spot, radians; sun: cutoff = cosine of the sun's half angle */
    float radius;          /* sphere: object-space radius */
    /* what the non-uniform light selectors know of a finite light
     * (Light::position / direction / computeFlux, light/Light.h:22-23;
     * AreaLight.cpp:46-112, PointLight.cpp:12-30, SpotLight.cpp:12-38) */
    float select_position[3];
    float select_direction[3];
    int32_t select_has_direction;
    float select_flux;     /* mean of the light's power colour */
} igx_light;

/* ---- camera / technique ------------------------------------------------ */
typedef struct igx_camera {
    float eye[3], dir[3], up[3];
    float fov;             /* radians */
    int32_t vertical_fov;  /* 1: fov is vertical (compute_scale_from_vfov) */
    float aspect;          /* <= 0: use film width / height */
    float near_clip, far_clip;
} igx_camera;

/* light selection for next-event estimation (LoaderLight::generateLightSelector,
 * LoaderLight.cpp:423-453; light/light_selector.art) */
enum { IGX_SELECT_UNIFORM = 0, IGX_SELECT_SIMPLE = 1, IGX_SELECT_HIERARCHY = 2 };

typedef struct igx_technique {
    int32_t max_depth;     /* PathTechnique.cpp:11, default 64 */
    int32_t min_depth;     /* default 2 */
    float clamp;           /* <= 0: no clamping */
    int32_t nee;           /* next-event estimation on */
    int32_t light_selector;/* IGX_SELECT_*: "uniform" (default), "simple" (flux CDF), "hierarchy" (light BVH) */
    int32_t aov_mis;       /* PathTechnique.cpp:16: the "Direct Weights" / "NEE Weights" AOVs (igx_get_aov) */
} igx_technique;

typedef struct igx_scene_desc {
    int32_t film_width, film_height;
    igx_camera camera;
    igx_technique technique;
    uint32_t num_meshes;    const igx_mesh* meshes;
    uint32_t num_shapes;    const igx_shape* shapes;
    uint32_t num_entities;  const igx_entity* entities;
    uint32_t num_materials; const igx_material* materials;
    uint32_t num_lights;    const igx_light* lights;
    float scene_bbox_min[3], scene_bbox_max[3];
} igx_scene_desc;

/* ---- loader C-ABI (stand-in for the reference's Loader, src/runtime/loader) */
typedef struct igx_scene igx_scene;

/* Load a scene JSON file (Ignis schema subset).  Relative mesh paths resolve
 * against the directory of `path`.  Returns NULL and fills err (if given) on
 * failure.  Mirrors SceneParser::loadFromFile + Loader::load
 * (src/runtime/Runtime.cpp:143-163, 202-290). */
igx_scene* igx_scene_load_file(const char* path, char* err, size_t err_len);
/* Same, from a JSON string; `base_dir` resolves external files (may be NULL). */
igx_scene* igx_scene_load_string(const char* json, const char* base_dir, char* err, size_t err_len);
const igx_scene_desc* igx_scene_get_desc(const igx_scene* scene);
void igx_scene_free(igx_scene* scene);
/* Names of a scene from igx_scene_load_*, for bindings that re-index its
 * shading tables by the reference loader's ids: the
 * material id of (BSDF name, emissive entity name or NULL/"" for a shared
 * material, LoaderContext::Material, LoaderContext.h:19-27), -1 if absent;
 * the name of entity `entity`, NULL if out of range (or for scenes built by
 * igx_scene_from_database, which carry no names). */
int32_t igx_scene_find_material(const igx_scene* scene, const char* bsdf, const char* emissive_entity);
const char* igx_scene_entity_name(const igx_scene* scene, uint32_t entity);

/* ---- in-memory scenes: the reference's IG::Scene object model ------------
 * Runtime::loadFromString / loadFromScene parse (or receive) an IG::Scene and
 * call load({}, scene) without a file (Runtime.cpp:164-199).  A binding that
 * holds such a `const Scene*` (Scene.h: technique, camera, film and named
 * textures / bsdfs / shapes / lights / media / entities, each a SceneObject
 * with a plugin type and SceneProperty values, SceneObject.h, SceneProperty.h)
 * rebuilds it here object by object and property by property, and
 * igx_scene_from_objects reads it with the same semantics as the JSON loader
 * -- no file and no second parse.  An in-memory JSON string goes through
 * igx_scene_load_string. */
typedef struct igx_objscene igx_objscene;
/* SceneObject::Type (SceneObject.h:10-22) */
enum {
    IGX_OBJ_BSDF = 0, IGX_OBJ_CAMERA = 1, IGX_OBJ_ENTITY = 2, IGX_OBJ_FILM = 3, IGX_OBJ_LIGHT = 4, IGX_OBJ_MEDIUM = 5,
    IGX_OBJ_SHAPE = 6, IGX_OBJ_TECHNIQUE = 7, IGX_OBJ_TEXTURE = 8, IGX_OBJ_PARAMETER = 9
};
/* SceneProperty::Type (SceneProperty.h:17-28) and the data each takes:
 * BOOL, INTEGER: int32_t[1]; NUMBER: float[1]; STRING: a NUL-terminated char*;
 * TRANSFORM: float[16], row-major 4x4 (Eigen's Transformf::matrix() is
 * column-major: transpose it); VECTOR2 float[2]; VECTOR3 float[3];
 * INTEGER_ARRAY int32_t[count]; NUMBER_ARRAY float[count] */
enum {
    IGX_PROP_BOOL = 1, IGX_PROP_INTEGER = 2, IGX_PROP_NUMBER = 3, IGX_PROP_STRING = 4, IGX_PROP_TRANSFORM = 5,
    IGX_PROP_VECTOR2 = 6, IGX_PROP_VECTOR3 = 7, IGX_PROP_INTEGER_ARRAY = 8, IGX_PROP_NUMBER_ARRAY = 9
};
/* `base_dir` resolves relative file names (mesh files) of objects added
 * without their own directory (SceneObject::baseDir); may be NULL. */
igx_objscene* igx_objscene_create(const char* base_dir);
void igx_objscene_free(igx_objscene* scene);
/* Add an object (Scene::addBSDF / setCamera / ...): a named object replaces
 * one of the same type and name; camera, film and technique ignore `name` and
 * replace the previous one.  `base_dir` may be NULL.  Returns the object's
 * handle (>= 0) or -1 for an unknown type. */
int32_t igx_objscene_add(igx_objscene* scene, int32_t object_type, const char* plugin_type, const char* name,
                         const char* base_dir);
/* SceneObject::setProperty: 0 on success, -1 for a bad handle, type or data. */
int32_t igx_objscene_set_property(igx_objscene* scene, int32_t object, const char* key, int32_t property_type,
                                  const void* data, uint64_t count);
/* Load the object scene like igx_scene_load_string loads a JSON scene.
 * Returns NULL and fills err on unsupported or malformed objects. */
igx_scene* igx_scene_from_objects(const igx_objscene* scene, char* err, size_t err_len);

/* ---- the reference's SceneDatabase as plain C (Device::assignScene seam) --
 * IG::Runtime hands its device a `SceneDatabase*` (Runtime.cpp:477-485,
 * Device.h:25-30; table/SceneDatabase.h:13-20).  A binding passes views of the
 * tables it holds; igx_scene_from_database turns them into an igx_scene whose
 * desc equals what igx_scene_load_file builds from the same scene file. */

/* DynTable lookup entry (table/DynTable.h:6-10), 16 bytes */
typedef struct igx_lookup_entry {
    uint32_t type_id;  /* ShapeProvider::id() for the "shapes" table */
    uint32_t flags;
    uint64_t offset;   /* byte offset of the record in the table data */
} igx_lookup_entry;

/* one DynTable / FixTable / SceneBVH byte array */
typedef struct igx_db_table {
    const uint8_t* data;
    uint64_t bytes;
    const igx_lookup_entry* lookups; /* DynTable only (NULL for a FixTable) */
    uint64_t count;                  /* DynTable: lookup count; FixTable: entryCount() */
} igx_db_table;

typedef struct igx_database_view {
    /* FixTables["entities"]: 36 x 4 B per entity, column-major toLocal 3x4,
     * toGlobal 3x4, normal 3x3, u32 shape_id, u32 material_id, pad
     * (LoaderEntity.cpp:155-162) */
    igx_db_table entities;
    /* DynTables["shapes"]: trimesh records (TriMeshProvider.cpp:583-598:
     * u32 faces, vertices, normals, texcoords; bbox min.xyz, 0, max.xyz, 0;
     * vertices and normals 16 B each; indices 4 x u32 per face; texcoords 8 B
     * each) and sphere records (SphereProvider.cpp:40-47: origin.xyz, radius) */
    igx_db_table shapes;
    uint32_t trimesh_type_id;  /* lookup type_id of the trimesh provider */
    uint32_t sphere_type_id;   /* lookup type_id of the sphere provider */
    /* FixTables["trimesh_primbvh"]: GPU-target BLAS blobs (TriMeshProvider.cpp:
     * 361-369); may be empty (igx then builds the BLAS itself) */
    igx_db_table trimesh_primbvh;
    /* SceneBVHs[provider].Leaves: EntityLeaf1 records (96 B, traversal/bvh.art:
     * 52-61; SceneBVHAdapter.h:88-104) of every provider's TLAS.  They carry the
     * entity visibility flags (LoaderEntity.cpp:120-128) and, in user[0..1],
     * the float offset of the entity's BLAS in trimesh_primbvh */
    const igx_db_table* scene_bvh_leaves;
    uint32_t num_scene_bvhs;
    float scene_bbox_min[3], scene_bbox_max[3]; /* SceneDatabase::SceneBBox */
} igx_database_view;

/* The part of a scene the reference compiles into shader code instead of
 * tables (the TechniqueVariantShaderSet handed to Device::render, Device.h:52):
 * film, camera, technique, the material of every material id
 * (LoaderContext::Materials order, LoaderEntity.cpp:42-103) and the lights
 * (area lights name their entity by its index in the entities table). */
typedef struct igx_shading_view {
    int32_t film_width, film_height;
    igx_camera camera;
    igx_technique technique;
    uint32_t num_materials; const igx_material* materials;
    uint32_t num_lights;    const igx_light* lights;
} igx_shading_view;

/* Build a scene from the reference's tables plus the shading view.  Plane
 * shapes are recognised from the mesh records (TriMesh::getAsPlane, as
 * TriMeshProvider.cpp:562 does); entity world boxes follow
 * BoundingBox::transformed (LoaderEntity.cpp:141).  With a non-empty
 * trimesh_primbvh, every trimesh shape carries its reference BLAS (ref_bvh),
 * which igx_upload_scene then uses instead of building one (option
 * "rebuild_bvh" = 1 ignores it).  Returns NULL and fills err on malformed
 * tables (sizes, offsets, ids out of range). */
igx_scene* igx_scene_from_database(const igx_database_view* db, const igx_shading_view* shading, char* err,
                                   size_t err_len);

/* Write a linear RGB image (row-major, 3 floats per pixel, each multiplied by
 * `scale`, e.g. 1/iteration count) as an uncompressed float OpenEXR file with
 * `channels` = 3 (RGB) or 4 (RGB + alpha 1).  Replaces Image::save
 * (src/runtime/Image.h:92-101) for the framebuffer output.  0 on success. */
int igx_write_exr(const char* path, const float* rgb, int32_t width, int32_t height, int32_t channels, float scale);

#ifdef __cplusplus
}
#endif
#endif
