"""ctypes binding of the igx C-ABI (include/igx.h, include/igx_scene.h).

The shared library is built in-tree (``make -C ignis-masterthesis_amd``) and is
loaded from the package's parent directory.  There is no fallback: if the
library is missing, importing the runtime raises, so nothing silently runs on
the CPU.
"""
import ctypes as C
import os

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# IGX_LIB_PATH: a variant build of the same library (dev A/B runs, tools/ab_libs.sh)
LIB_PATH = os.environ.get("IGX_LIB_PATH") or os.path.join(os.path.dirname(_PKG_DIR), "libigx.so")

# ---- igx_scene.h ----------------------------------------------------------


class Mesh(C.Structure):
    _fields_ = [("num_vertices", C.c_uint32), ("num_faces", C.c_uint32),
                ("vertices", C.POINTER(C.c_float)), ("normals", C.POINTER(C.c_float)),
                ("texcoords", C.POINTER(C.c_float)), ("indices", C.POINTER(C.c_uint32))]


class Shape(C.Structure):
    _fields_ = [("type", C.c_int32), ("mesh", C.c_int32), ("sphere", C.c_float * 4),
                ("bbox_min", C.c_float * 3), ("bbox_max", C.c_float * 3), ("is_plane", C.c_int32),
                ("plane_origin", C.c_float * 3), ("plane_x", C.c_float * 3), ("plane_y", C.c_float * 3),
                ("plane_tex", C.c_float * 8), ("ref_bvh", C.c_void_p), ("ref_bvh_bytes", C.c_uint64)]


class Entity(C.Structure):
    _fields_ = [("shape", C.c_int32), ("material", C.c_int32), ("flags", C.c_uint32),
                ("to_global", C.c_float * 12), ("to_local", C.c_float * 12), ("normal", C.c_float * 9),
                ("bbox_min", C.c_float * 3), ("bbox_max", C.c_float * 3)]


class Material(C.Structure):
    _fields_ = [("bsdf_type", C.c_int32), ("light", C.c_int32), ("thin", C.c_int32), ("distribution", C.c_int32),
                ("kd", C.c_float * 3), ("ks", C.c_float * 3), ("kt", C.c_float * 3),
                ("ext_ior", C.c_float), ("int_ior", C.c_float), ("eta", C.c_float * 3), ("kappa", C.c_float * 3),
                ("alpha_u", C.c_float), ("alpha_v", C.c_float), ("diffuse_alpha", C.c_float), ("pad", C.c_float),
                ("ior", C.c_float), ("diffuse_transmission", C.c_float), ("specular_transmission", C.c_float),
                ("specular_tint", C.c_float), ("flatness", C.c_float), ("metallic", C.c_float), ("sheen", C.c_float),
                ("sheen_tint", C.c_float), ("clearcoat", C.c_float), ("clearcoat_gloss", C.c_float),
                ("clearcoat_roughness", C.c_float), ("clearcoat_top_only", C.c_int32),
                ("texture", C.c_int32), ("tex_scale", C.c_float), ("tex_kd1", C.c_float * 3)]


# igx_light.type (include/igx_scene.h)
LIGHT_PLANE, LIGHT_ENV, LIGHT_POINT, LIGHT_SPOT, LIGHT_DIRECTIONAL, LIGHT_SUN, LIGHT_SPHERE, LIGHT_MESH = range(1, 9)


class Light(C.Structure):
    _fields_ = [("type", C.c_int32), ("entity", C.c_int32), ("radiance", C.c_float * 3),
                ("origin", C.c_float * 3), ("x_axis", C.c_float * 3), ("y_axis", C.c_float * 3),
                ("normal", C.c_float * 3), ("area", C.c_float), ("cutoff", C.c_float), ("falloff", C.c_float),
                ("radius", C.c_float), ("select_position", C.c_float * 3), ("select_direction", C.c_float * 3),
                ("select_has_direction", C.c_int32), ("select_flux", C.c_float)]


class Camera(C.Structure):
    _fields_ = [("eye", C.c_float * 3), ("dir", C.c_float * 3), ("up", C.c_float * 3), ("fov", C.c_float),
                ("vertical_fov", C.c_int32), ("aspect", C.c_float), ("near_clip", C.c_float), ("far_clip", C.c_float)]


class Technique(C.Structure):
    _fields_ = [("max_depth", C.c_int32), ("min_depth", C.c_int32), ("clamp", C.c_float), ("nee", C.c_int32),
                ("light_selector", C.c_int32), ("aov_mis", C.c_int32)]


class SceneDesc(C.Structure):
    _fields_ = [("film_width", C.c_int32), ("film_height", C.c_int32), ("camera", Camera),
                ("technique", Technique),
                ("num_meshes", C.c_uint32), ("meshes", C.POINTER(Mesh)),
                ("num_shapes", C.c_uint32), ("shapes", C.POINTER(Shape)),
                ("num_entities", C.c_uint32), ("entities", C.POINTER(Entity)),
                ("num_materials", C.c_uint32), ("materials", C.POINTER(Material)),
                ("num_lights", C.c_uint32), ("lights", C.POINTER(Light)),
                ("scene_bbox_min", C.c_float * 3), ("scene_bbox_max", C.c_float * 3)]


class LookupEntry(C.Structure):
    _fields_ = [("type_id", C.c_uint32), ("flags", C.c_uint32), ("offset", C.c_uint64)]


class DbTable(C.Structure):
    _fields_ = [("data", C.c_void_p), ("bytes", C.c_uint64), ("lookups", C.POINTER(LookupEntry)), ("count", C.c_uint64)]


class DatabaseView(C.Structure):
    _fields_ = [("entities", DbTable), ("shapes", DbTable), ("trimesh_type_id", C.c_uint32),
                ("sphere_type_id", C.c_uint32), ("trimesh_primbvh", DbTable),
                ("scene_bvh_leaves", C.POINTER(DbTable)), ("num_scene_bvhs", C.c_uint32),
                ("scene_bbox_min", C.c_float * 3), ("scene_bbox_max", C.c_float * 3)]


class ShadingView(C.Structure):
    _fields_ = [("film_width", C.c_int32), ("film_height", C.c_int32), ("camera", Camera), ("technique", Technique),
                ("num_materials", C.c_uint32), ("materials", C.POINTER(Material)),
                ("num_lights", C.c_uint32), ("lights", C.POINTER(Light))]


# ---- igx.h ----------------------------------------------------------------

class RenderParams(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("spi", C.c_int32), ("iteration", C.c_int32),
                ("frame", C.c_int32), ("seed", C.c_int32), ("tile_size", C.c_int32), ("tile_offset", C.c_int32),
                ("tile_stride", C.c_int32), ("num_rays", C.c_int32), ("rays", C.POINTER(C.c_float))]


class Stats(C.Structure):
    _fields_ = [("camera_rays", C.c_uint64), ("bounce_rays", C.c_uint64), ("shadow_rays", C.c_uint64),
                ("iterations", C.c_uint64), ("launches_extend", C.c_uint64), ("launches_shadow", C.c_uint64),
                ("ms_extend", C.c_double), ("ms_shadow", C.c_double), ("ms_generate", C.c_double),
                ("ms_resolve", C.c_double), ("ms_render", C.c_double),
                ("node_visits", C.c_uint64), ("leaf_visits", C.c_uint64), ("tri_tests", C.c_uint64),
                ("blas_enters", C.c_uint64), ("shadow_node_visits", C.c_uint64),
                ("shadow_leaf_visits", C.c_uint64), ("shadow_tri_tests", C.c_uint64),
                ("shadow_blas_enters", C.c_uint64), ("shaded_hits", C.c_uint64),
                ("launches_finish", C.c_uint64), ("ms_finish", C.c_double), ("tail_bounce_rays", C.c_uint64),
                ("tail_shadow_rays", C.c_uint64), ("bvh_depth", C.c_int32), ("stack_entries", C.c_int32),
                ("extend_rays", C.c_uint64), ("extend_paths_out", C.c_uint64),
                ("launches_trace", C.c_uint64), ("ms_trace", C.c_double),
                ("wave_node_iters", C.c_uint64), ("wave_leaf_iters", C.c_uint64),
                ("shadow_wave_node_iters", C.c_uint64), ("shadow_wave_leaf_iters", C.c_uint64),
                ("bvh_width", C.c_int32), ("node_bytes", C.c_int32),
                ("lds_scene_bytes", C.c_int32), ("shadow_blocks_per_cu", C.c_int32),
                ("table_bytes", C.c_uint64), ("shading_bytes", C.c_uint64),
                ("extend_cycles_load", C.c_uint64), ("extend_cycles_trace", C.c_uint64),
                ("extend_cycles_shade", C.c_uint64), ("extend_cycles_store", C.c_uint64),
                ("slot_bytes", C.c_uint64), ("treelet_nodes", C.c_int32 * 4),
                ("extend_class_cycles", C.c_uint64 * 8), ("extend_class_groups", C.c_uint64 * 4),
                ("extend_class_node_iters", C.c_uint64 * 4), ("extend_class_node_visits", C.c_uint64 * 4),
                ("shadow_class_groups", C.c_uint64 * 2), ("shadow_class_node_iters", C.c_uint64 * 2),
                ("shadow_class_node_visits", C.c_uint64 * 2), ("shadow_class_cycles", C.c_uint64 * 2),
                ("shadow_class_occluded", C.c_uint64 * 2), ("tlas_node_visits", C.c_uint64),
                ("hot_node_visits", C.c_uint64 * 3), ("extend_class_shade_cycles", C.c_uint64 * 16),
                ("shadow_class_rays", C.c_uint64 * 2)]

    def as_dict(self):
        return {name: (list(getattr(self, name)) if isinstance(getattr(self, name), C.Array) else getattr(self, name))
                for name, _ in self._fields_}


# every symbol include/igx.h and include/igx_scene.h declare
EXPORTED_SYMBOLS = [
    "igx_scene_load_file", "igx_scene_load_string", "igx_scene_get_desc", "igx_scene_free", "igx_write_exr",
    "igx_scene_from_database", "igx_scene_find_material", "igx_scene_entity_name",
    "igx_create", "igx_destroy", "igx_last_error", "igx_version", "igx_set_option", "igx_upload_scene",
    "igx_render", "igx_get_framebuffer", "igx_framebuffer_device_ptr", "igx_get_aov", "igx_aov_device_ptr",
    "igx_pack_tiles", "igx_clear", "igx_get_stats", "igx_reset_stats", "igx_trace_hits", "igx_trace_occlusion", "igx_synchronize", "igx_wait_ready",
    "igx_render_iterations", "igx_objscene_create", "igx_objscene_free", "igx_objscene_add",
    "igx_objscene_set_property", "igx_scene_from_objects", "igx_set_camera",
]

_lib = None


def lib():
    """Load libigx.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libigx.so not found at {LIB_PATH}; build it with `make -C ignis-masterthesis_amd`")
    L = C.CDLL(LIB_PATH)
    vp = C.c_void_p
    L.igx_scene_load_file.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t]
    L.igx_scene_load_file.restype = vp
    L.igx_scene_load_string.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_size_t]
    L.igx_scene_load_string.restype = vp
    L.igx_scene_from_database.argtypes = [C.POINTER(DatabaseView), C.POINTER(ShadingView), C.c_char_p, C.c_size_t]
    L.igx_scene_from_database.restype = vp
    L.igx_scene_find_material.argtypes = [vp, C.c_char_p, C.c_char_p]
    L.igx_scene_find_material.restype = C.c_int32
    L.igx_scene_entity_name.argtypes = [vp, C.c_uint32]
    L.igx_scene_entity_name.restype = C.c_char_p
    L.igx_scene_get_desc.argtypes = [vp]
    L.igx_scene_get_desc.restype = C.POINTER(SceneDesc)
    L.igx_scene_free.argtypes = [vp]
    L.igx_scene_free.restype = None
    L.igx_objscene_create.argtypes = [C.c_char_p]
    L.igx_objscene_create.restype = vp
    L.igx_objscene_free.argtypes = [vp]
    L.igx_objscene_free.restype = None
    L.igx_objscene_add.argtypes = [vp, C.c_int32, C.c_char_p, C.c_char_p, C.c_char_p]
    L.igx_objscene_add.restype = C.c_int32
    L.igx_objscene_set_property.argtypes = [vp, C.c_int32, C.c_char_p, C.c_int32, C.c_void_p, C.c_uint64]
    L.igx_objscene_set_property.restype = C.c_int32
    L.igx_scene_from_objects.argtypes = [vp, C.c_char_p, C.c_size_t]
    L.igx_scene_from_objects.restype = vp
    L.igx_set_camera.argtypes = [vp, C.POINTER(Camera)]
    L.igx_write_exr.argtypes = [C.c_char_p, C.POINTER(C.c_float), C.c_int32, C.c_int32, C.c_int32, C.c_float]
    L.igx_write_exr.restype = C.c_int
    L.igx_create.argtypes = [C.c_int, C.POINTER(vp)]
    L.igx_destroy.argtypes = [vp]
    L.igx_last_error.argtypes = [vp]
    L.igx_last_error.restype = C.c_char_p
    L.igx_version.argtypes = []
    L.igx_version.restype = C.c_char_p
    L.igx_set_option.argtypes = [vp, C.c_char_p, C.c_int64]
    L.igx_upload_scene.argtypes = [vp, vp]
    L.igx_render.argtypes = [vp, C.POINTER(RenderParams)]
    L.igx_render_iterations.argtypes = [vp, C.POINTER(RenderParams), C.c_int32]
    L.igx_get_framebuffer.argtypes = [vp, C.POINTER(C.c_float), C.c_size_t, C.POINTER(C.c_uint64)]
    L.igx_framebuffer_device_ptr.argtypes = [vp, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
    L.igx_get_aov.argtypes = [vp, C.c_char_p, C.POINTER(C.c_float), C.c_size_t, C.POINTER(C.c_uint64)]
    L.igx_aov_device_ptr.argtypes = [vp, C.c_char_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
    L.igx_pack_tiles.argtypes = [vp, C.POINTER(RenderParams), C.c_void_p, C.c_size_t]
    L.igx_clear.argtypes = [vp]
    L.igx_synchronize.argtypes = [vp]
    L.igx_wait_ready.argtypes = [vp]
    L.igx_get_stats.argtypes = [vp, C.POINTER(Stats)]
    L.igx_reset_stats.argtypes = [vp]
    L.igx_trace_hits.argtypes = [vp, C.POINTER(C.c_float), C.c_int32, C.c_uint32, C.POINTER(C.c_int32),
                                 C.POINTER(C.c_float)]
    L.igx_trace_occlusion.argtypes = [vp, C.POINTER(C.c_float), C.c_int32, C.c_uint32, C.POINTER(C.c_int32)]
    for name in ["igx_create", "igx_destroy", "igx_set_option", "igx_upload_scene", "igx_render", "igx_render_iterations",
                 "igx_get_framebuffer", "igx_framebuffer_device_ptr", "igx_get_aov", "igx_aov_device_ptr",
                 "igx_pack_tiles", "igx_clear",
                 "igx_synchronize", "igx_wait_ready", "igx_get_stats", "igx_reset_stats", "igx_trace_hits", "igx_trace_occlusion"]:
        getattr(L, name).restype = C.c_int
    _lib = L
    return L
