"""ignis_amd — Python face of the MI355X wavefront path-tracing device.

Mirrors the reference's Python module surface used by its integration tests
(src/frontend/python/runtime.cpp:178-260; src/tests/integrator/common/__init__.py:68-90):

    opts = ignis_amd.RuntimeOptions.makeDefault()
    with ignis_amd.loadFromString(json_text, opts) as runtime:
        runtime.step()
        img = runtime.getFramebufferForHost() / runtime.IterationCount

Semantics follow IG::Runtime (src/runtime/Runtime.cpp): SPI defaults to the
reference's GPU recommendation (8 for a 1000^2 film, Runtime.cpp:61-69), each
step() renders one iteration (Runtime::step, Runtime.cpp:292-319) and the
framebuffer holds sum(colour)/spi per pixel until cleared.
"""
import ctypes as C
import json
import math
import os

import numpy as np

from . import _native
from ._native import EXPORTED_SYMBOLS, LIB_PATH, RenderParams, Stats, lib

__all__ = ["RuntimeOptions", "Scene", "Runtime", "loadFromFile", "loadFromString", "version",
           "EXPORTED_SYMBOLS", "LIB_PATH", "IgxError"]


class IgxError(RuntimeError):
    pass


def version():
    return lib().igx_version().decode()


def write_exr(path, rgb, scale=1.0, alpha=False):
    """Write a (H, W, 3) float image as an uncompressed float OpenEXR file
    (Image::save, src/runtime/Image.h:92-101)."""
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    h, w = rgb.shape[0], rgb.shape[1]
    rc = _native.lib().igx_write_exr(os.fsencode(path), rgb.ctypes.data_as(C.POINTER(C.c_float)), w, h, 4 if alpha else 3,
                                      float(scale))
    if rc != 0:
        raise IgxError(f"cannot write EXR {path} (code {rc})")


def recommend_spi(width, height, interactive=False):
    """Runtime.cpp:61-69 for a GPU target."""
    spi_f = 8
    if interactive:
        spi_f //= 2
    spi = math.ceil(spi_f / ((width / 1000.0) * (height / 1000.0)))
    return max(1, min(64, spi))


class RuntimeOptions:
    """Subset of IG::RuntimeOptions (src/runtime/RuntimeSettings.h:16-62)."""

    def __init__(self):
        self.Device = 0          # HIP device ordinal (--gpu-device)
        self.SPI = 0             # 0 = recommended
        self.Seed = 0
        self.AcquireStats = False
        self.OverrideFilmSize = (0, 0)
        self.Capacity = 0        # paths in flight; 0 = whole iteration (<= 16M)

    @staticmethod
    def makeDefault():
        return RuntimeOptions()


class Scene:
    """A loaded scene (owner of the igx_scene handle)."""

    def __init__(self, handle):
        self._h = handle

    @staticmethod
    def from_file(path):
        err = C.create_string_buffer(2048)
        h = lib().igx_scene_load_file(os.fsencode(path), err, len(err))
        if not h:
            raise IgxError(err.value.decode())
        return Scene(h)

    @staticmethod
    def from_string(text, base_dir=None):
        if isinstance(text, dict):
            text = json.dumps(text)
        err = C.create_string_buffer(2048)
        h = lib().igx_scene_load_string(text.encode(), os.fsencode(base_dir) if base_dir else None, err, len(err))
        if not h:
            raise IgxError(err.value.decode())
        return Scene(h)

    @staticmethod
    def from_objects(objects):
        """igx_scene_from_objects: a scene built object by object
        (`ObjectScene`, the reference's in-memory IG::Scene)."""
        err = C.create_string_buffer(2048)
        h = lib().igx_scene_from_objects(objects._h, err, len(err))
        if not h:
            raise IgxError(err.value.decode())
        return Scene(h)

    @staticmethod
    def from_database(db, shading):
        """igx_scene_from_database: the reference's SceneDatabase tables
        (`_native.DatabaseView`) plus the shading tables (`_native.ShadingView`);
        the caller keeps the viewed buffers alive for the call."""
        err = C.create_string_buffer(2048)
        h = lib().igx_scene_from_database(C.byref(db), C.byref(shading), err, len(err))
        if not h:
            raise IgxError(err.value.decode())
        return Scene(h)

    @property
    def desc_ptr(self):
        """Raw `const igx_scene_desc*` (for C consumers such as the oracle)."""
        return C.cast(lib().igx_scene_get_desc(self._h), C.c_void_p)

    @property
    def desc(self):
        return lib().igx_scene_get_desc(self._h).contents

    @property
    def film_size(self):
        d = self.desc
        return d.film_width, d.film_height

    def close(self):
        if self._h:
            lib().igx_scene_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ObjectScene:
    """The reference's in-memory scene (IG::Scene: technique, camera, film and
    named bsdfs / shapes / lights / entities / textures / media, each a
    SceneObject of SceneProperty values) built through the igx_objscene_* C-ABI,
    the way a binding forwards the `const Scene*` that Runtime::loadFromScene
    receives (Runtime.cpp:183-199)."""

    OBJ = {"bsdfs": 0, "camera": 1, "entities": 2, "film": 3, "lights": 4, "media": 5, "shapes": 6, "technique": 7,
           "textures": 8, "parameters": 9}
    BOOL, INTEGER, NUMBER, STRING, TRANSFORM, VECTOR2, VECTOR3, INTEGER_ARRAY, NUMBER_ARRAY = range(1, 10)

    def __init__(self, base_dir=None):
        self._h = lib().igx_objscene_create(os.fsencode(base_dir) if base_dir else None)

    def add(self, category, plugin_type, name=None, base_dir=None):
        h = lib().igx_objscene_add(self._h, self.OBJ[category], plugin_type.encode(), name.encode() if name else None,
                                   os.fsencode(base_dir) if base_dir else None)
        if h < 0:
            raise IgxError(f"igx_objscene_add({category}, {plugin_type}, {name}) refused")
        return h

    def set(self, obj, key, ptype, value):
        if ptype == self.STRING:
            buf = C.create_string_buffer(value.encode())
            data, n = C.cast(buf, C.c_void_p), 1
        elif ptype in (self.BOOL, self.INTEGER, self.INTEGER_ARRAY):
            vals = [int(v) for v in (value if isinstance(value, (list, tuple)) else [value])]
            buf = (C.c_int32 * max(1, len(vals)))(*vals)
            data, n = C.cast(buf, C.c_void_p), len(vals)
        else:
            vals = [float(v) for v in (value if isinstance(value, (list, tuple)) else [value])]
            buf = (C.c_float * max(1, len(vals)))(*vals)
            data, n = C.cast(buf, C.c_void_p), len(vals)
        if lib().igx_objscene_set_property(self._h, obj, key.encode(), ptype, data, n) != 0:
            raise IgxError(f"igx_objscene_set_property({key}) refused")

    def set_value(self, obj, key, v):
        """A JSON value typed as the reference parser types it (getProperty, Parser.cpp:281-318)."""
        if isinstance(v, bool):
            self.set(obj, key, self.BOOL, int(v))
        elif isinstance(v, str):
            self.set(obj, key, self.STRING, v)
        elif isinstance(v, int):
            self.set(obj, key, self.INTEGER, v)
        elif isinstance(v, float):
            self.set(obj, key, self.NUMBER, v)
        elif isinstance(v, list):
            if len(v) == 2:
                self.set(obj, key, self.VECTOR2, v)
            elif len(v) == 3:
                self.set(obj, key, self.VECTOR3, v)
            elif len(v) in (9, 12, 16):
                m = [[1.0 if i == j else 0.0 for j in range(4)] for i in range(4)]
                for i in range(3 if len(v) != 16 else 4):
                    for j in range(3 if len(v) == 9 else 4):
                        m[i][j] = float(v[i * (3 if len(v) == 9 else 4) + j])
                self.set(obj, key, self.TRANSFORM, [x for row in m for x in row])
            else:
                raise IgxError(f"property '{key}': an array of {len(v)} is not a scene property")
        elif isinstance(v, dict) and "values" in v:
            ints = str(v.get("type", "")) in ("int", "integer")
            self.set(obj, key, self.INTEGER_ARRAY if ints else self.NUMBER_ARRAY, v["values"])
        else:
            raise IgxError(f"property '{key}': unsupported value {v!r}")

    @staticmethod
    def from_dict(scene, base_dir=None):
        """Every object of a scene dict (the JSON schema), as a binding would
        forward the parsed IG::Scene's objects."""
        o = ObjectScene(base_dir)
        for cat in ("technique", "camera", "film"):
            if cat in scene:
                d = scene[cat]
                h = o.add(cat, d.get("type", ""))
                for k, v in d.items():
                    if k != "type":
                        o.set_value(h, k, v)
        for cat in ("textures", "bsdfs", "shapes", "lights", "media", "entities"):
            for d in scene.get(cat, []):
                h = o.add(cat, d.get("type", ""), d["name"])
                for k, v in d.items():
                    if k not in ("type", "name"):
                        o.set_value(h, k, v)
        return o

    def close(self):
        if self._h:
            lib().igx_objscene_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Device:
    """Thin owner of an igx_device handle (IG::Device, src/runtime/device/Device.h:14-74)."""

    def __init__(self, hip_device=0):
        self._lib = lib()
        h = C.c_void_p()
        st = self._lib.igx_create(int(hip_device), C.byref(h))
        if st != 0 or not h:
            raise IgxError(f"igx_create({hip_device}) failed with status {st}")
        self._h = h

    def _check(self, st):
        if st != 0:
            raise IgxError(self._lib.igx_last_error(self._h).decode())

    def set_option(self, key, value):
        self._check(self._lib.igx_set_option(self._h, key.encode(), int(value)))

    def upload(self, scene):
        self._check(self._lib.igx_upload_scene(self._h, scene.desc_ptr))

    def render(self, params):
        self._check(self._lib.igx_render(self._h, C.byref(params)))

    def set_camera(self, camera):
        """Replace the uploaded scene's camera (an N.Camera; igx_set_camera, as
        Runtime::setCameraOrientationParameter reaches the device through
        render's ParameterSet, Runtime.cpp:703-708)."""
        self._check(self._lib.igx_set_camera(self._h, C.byref(camera)))

    def render_iterations(self, params, count):
        """`count` consecutive iterations from params.iteration (igx_render_iterations)."""
        self._check(self._lib.igx_render_iterations(self._h, C.byref(params), int(count)))

    def framebuffer(self, count, name=None):
        """The film, or a named AOV (igx_get_aov: "Color", and with the
        technique's aov_mis "Direct Weights" / "NEE Weights")."""
        out = np.zeros(count, dtype=np.float32)
        it = C.c_uint64()
        if name is None:
            self._check(self._lib.igx_get_framebuffer(self._h, out.ctypes.data_as(C.POINTER(C.c_float)), count, C.byref(it)))
        else:
            self._check(self._lib.igx_get_aov(self._h, name.encode(), out.ctypes.data_as(C.POINTER(C.c_float)), count,
                                              C.byref(it)))
        return out, int(it.value)

    def framebuffer_device_ptr(self):
        p = C.c_void_p()
        n = C.c_size_t()
        self._check(self._lib.igx_framebuffer_device_ptr(self._h, C.byref(p), C.byref(n)))
        return p.value, n.value

    def pack_tiles(self, params, dst_ptr, count):
        self._check(self._lib.igx_pack_tiles(self._h, C.byref(params), C.c_void_p(dst_ptr), count))

    def clear(self):
        self._check(self._lib.igx_clear(self._h))

    def synchronize(self):
        self._check(self._lib.igx_synchronize(self._h))

    def wait_ready(self):
        """igx_wait_ready: the handle's queued chunks are in their late bounces."""
        self._check(self._lib.igx_wait_ready(self._h))

    def stats(self):
        s = Stats()
        self._check(self._lib.igx_get_stats(self._h, C.byref(s)))
        return s.as_dict()

    def reset_stats(self):
        self._check(self._lib.igx_reset_stats(self._h))

    def trace_hits(self, rays, flags=0x1):
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
        n = rays.shape[0]
        ep = np.zeros((n, 2), dtype=np.int32)
        tuv = np.zeros((n, 3), dtype=np.float32)
        self._check(self._lib.igx_trace_hits(self._h, rays.ctypes.data_as(C.POINTER(C.c_float)), n, flags,
                                             ep.ctypes.data_as(C.POINTER(C.c_int32)),
                                             tuv.ctypes.data_as(C.POINTER(C.c_float))))
        return ep, tuv

    def trace_occlusion(self, rays, flags=0x8):
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
        n = rays.shape[0]
        occ = np.zeros(n, dtype=np.int32)
        self._check(self._lib.igx_trace_occlusion(self._h, rays.ctypes.data_as(C.POINTER(C.c_float)), n, flags,
                                                  occ.ctypes.data_as(C.POINTER(C.c_int32))))
        return occ

    def close(self):
        if getattr(self, "_h", None):
            self._lib.igx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Runtime:
    """IG::Runtime restricted to the hot path (src/runtime/Runtime.h:19-198)."""

    def __init__(self, scene, opts=None):
        opts = opts or RuntimeOptions.makeDefault()
        self.scene = scene
        self.options = opts
        w, h = scene.film_size
        if opts.OverrideFilmSize[0] > 0:
            w, h = opts.OverrideFilmSize
        self.FilmWidth, self.FilmHeight = int(w), int(h)
        self.SamplesPerIteration = opts.SPI if opts.SPI > 0 else recommend_spi(self.FilmWidth, self.FilmHeight)
        self.Seed = opts.Seed
        self.device = Device(opts.Device)
        if opts.AcquireStats:
            self.device.set_option("timing", 1)
        if opts.Capacity:
            self.device.set_option("capacity", opts.Capacity)
        self.device.upload(scene)
        self._iteration = 0
        self._frame = 0
        self._fb_count = self.FilmWidth * self.FilmHeight * 3

    @property
    def IterationCount(self):
        return self._iters

    def _params(self, tile=None):
        p = RenderParams()
        p.width, p.height = self.FilmWidth, self.FilmHeight
        p.spi = self.SamplesPerIteration
        p.iteration = self._iteration
        p.frame = self._frame
        p.seed = self.Seed
        if tile is not None:
            p.tile_size, p.tile_offset, p.tile_stride = tile
        return p

    _iters = 0

    def step(self, tile=None):
        """Runtime::step: one iteration of SamplesPerIteration samples."""
        self.device.render(self._params(tile))
        self._iteration += 1
        self._iters += 1

    def getFramebufferForHost(self, name=""):
        """Runtime::getFramebufferForHost(name) (Runtime.cpp:417-435): the
        film ("" / "Color") or a named AOV of the technique."""
        fb, it = self.device.framebuffer(self._fb_count, name or None)
        self._iters = it
        return fb.reshape(self.FilmHeight, self.FilmWidth, 3)

    def clearFramebuffer(self):
        self.device.clear()
        self._iters = 0

    def reset(self):
        self.clearFramebuffer()
        self._iteration = 0

    def trace(self, rays):
        """Runtime::trace (Runtime.cpp:385-407): radiance per ray, one iteration."""
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
        p = self._params()
        p.num_rays = rays.shape[0]
        p.rays = rays.ctypes.data_as(C.POINTER(C.c_float))
        self.device.clear()
        self.device.render(p)
        fb, it = self.device.framebuffer(rays.shape[0] * 3)
        self.device.clear()
        return fb.reshape(-1, 3) / max(it, 1)

    def getStatistics(self):
        return self.device.stats()

    def close(self):
        self.device.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


def loadFromFile(path, opts=None):
    return Runtime(Scene.from_file(path), opts)


def loadFromString(text, opts=None, base_dir=None):
    return Runtime(Scene.from_string(text, base_dir), opts)
