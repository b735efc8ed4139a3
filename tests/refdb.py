"""Test-side writer of the reference's SceneDatabase byte layouts.

Serialises a scene igx's JSON loader produced into the tables the reference
loader hands its device (Runtime.cpp:477-485 -> Device::assignScene), following
the reference's writers, so the adapter igx_scene_from_database can be checked
against the direct-loader path:

* DynTables["shapes"]: DynTable::addLookup pads the data by a full alignment
  (16 B) even when it is already aligned, unless it is empty
  (table/DynTable.h:17-27).  Trimesh record (TriMeshProvider.cpp:583-598):
  u32 faces, vertices, normals, texcoords; bbox min.xyz, 0, max.xyz, 0;
  vertices and normals as Serializer::writeAligned(.., 16) = 12 B + 4 B pad
  (serialization/Serializer.inl:129-155); indices 4 x u32 per face; texcoords
  8 B each.  Sphere record (SphereProvider.cpp:40-47): origin.xyz, radius.
* FixTables["entities"]: addEntry(0), 36 x 4 B (LoaderEntity.cpp:155-162):
  toLocal 3x4, toGlobal 3x4, normal 3x3, all column-major; shape id, material
  id, pad.
* FixTables["trimesh_primbvh"]: addEntry(16) (same padding quirk,
  table/FixTable.h:15-24), offset = size / 4 after the pad
  (TriMeshProvider.cpp:361-369); blob = u32 node_count, tri_count, 0, 0;
  Node2[] (traversal/mapping_gpu.art:3-7: bounds lo_x, hi_x, lo_y, hi_y, lo_z,
  hi_z per child; child = inner index + 1, ~first Tri1, or 0 cut out,
  BvhNAdapter.h:121-148); Tri1[] (shapes/trimesh.art:107-114: v0, 0, e1 =
  v0 - v1, 0, e2 = v2 - v0, prim_id with bit 31 on the last of a leaf,
  TriBVHAdapter.h:148-158).  The tree here is a median split (the reference's
  madmann91/bvh SBVH is not available; topology does not change closest hits).
* SceneBVHs[provider].Leaves: EntityLeaf1 (96 B, traversal/bvh.art:52-61,
  SceneBVHAdapter.h:88-104): min.xyz, entity id (bit 31 = last of a leaf),
  max.xyz, shape id, local 3x4 column-major, flags, material id, user1/user2 =
  the BLAS offset in floats.  One leaf record per entity, in entity order.

This is test infrastructure, not product code.
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ignis-masterthesis_amd"))

from ignis_amd import _native as N  # noqa: E402

TRIMESH_PROVIDER_ID = 0  # ShapeProvider::id() (TriMeshProvider.h:13, SphereProvider.h:12)
SPHERE_PROVIDER_ID = 1


class Table:
    """DynTable / FixTable byte writer with the reference's padding rule."""

    def __init__(self):
        self.data = bytearray()
        self.lookups = []
        self.count = 0

    def add(self, alignment, type_id=None):
        if alignment and self.data:
            self.data += bytes(alignment - len(self.data) % alignment)  # a full pad when aligned (DynTable.h:20-23)
        if type_id is not None:
            self.lookups.append((type_id, 0, len(self.data)))
        self.count += 1
        return len(self.data)


def median_blas(v, faces, max_leaf=4):
    """Node2 + Tri1 blob of a median-split tree over the faces."""
    tri = v[faces]  # (n, 3, 3)
    n = len(faces)
    cen = tri.sum(axis=1)
    nodes, tris = [], []

    def box(ix):
        t = tri[ix].reshape(-1, 3)
        lo, hi = t.min(axis=0), t.max(axis=0)
        return [lo[0], hi[0], lo[1], hi[1], lo[2], hi[2]]

    def leaf(ix):
        ref = ~len(tris)
        for k, f in enumerate(ix):
            p0, p1, p2 = tri[f]
            prim = int(f) | (0x80000000 if k == len(ix) - 1 else 0)
            tris.append((p0, p0 - p1, p2 - p0, prim))
        return ref

    def node(ix):
        me = len(nodes)
        nodes.append([None, [0, 0]])
        b = box(ix)
        axis = int(np.argmax([b[1] - b[0], b[3] - b[2], b[5] - b[4]]))
        ix = ix[np.argsort(cen[ix, axis], kind="stable")]
        half = len(ix) // 2
        bounds = []
        for k, part in enumerate((ix[:half], ix[half:])):
            bounds += box(part)
            if len(part) <= max_leaf:
                nodes[me][1][k] = leaf(part)
            else:
                nodes[me][1][k] = len(nodes) + 1
                node(part)
        nodes[me][0] = bounds

    ix = np.arange(n)
    if n <= max_leaf:  # root leaf wrapped, sibling cut out (BvhNAdapter.h:94-98, 136-146)
        inf = np.float32(np.inf)
        nodes.append([box(ix) + [inf, -inf, inf, -inf, inf, -inf], [leaf(ix), 0]])
    else:
        node(ix)
    out = bytearray(np.array([len(nodes), len(tris), 0, 0], np.uint32).tobytes())
    for b, ch in nodes:
        out += np.array(b, np.float32).tobytes() + np.array(ch + [0, 0], np.int32).tobytes()
    for v0, e1, e2, prim in tris:
        rec = np.zeros(12, np.float32)
        rec[0:3], rec[4:7], rec[8:11] = v0, e1, e2
        r = rec.view(np.uint32)
        r[11] = prim & 0xFFFFFFFF
        out += rec.tobytes()
    return bytes(out)


def _col_major(rows, r, c):
    return np.array(rows, np.float32).reshape(r, c).T.reshape(-1)


class RefDatabase:
    """The reference tables of a loaded igx scene, plus ctypes views of them."""

    def __init__(self, scene, with_blas=True, max_leaf=4):
        d = scene.desc
        self.shapes = Table()
        self.entities = Table()
        self.primbvh = Table()
        blas_off = {}
        for s in range(d.num_shapes):
            sh = d.shapes[s]
            if sh.type == 1:
                off = self.shapes.add(16, SPHERE_PROVIDER_ID)
                self.shapes.data += np.array(list(sh.sphere), np.float32).tobytes()
                continue
            m = d.meshes[sh.mesh]
            nv, nf = m.num_vertices, m.num_faces
            v = np.ctypeslib.as_array(m.vertices, (nv * 3,)).reshape(nv, 3).copy()
            nrm = np.ctypeslib.as_array(m.normals, (nv * 3,)).reshape(nv, 3)
            tex = np.ctypeslib.as_array(m.texcoords, (nv * 2,)).reshape(nv, 2)
            faces = np.ctypeslib.as_array(m.indices, (nf * 3,)).reshape(nf, 3).astype(np.int64)
            off = self.shapes.add(16, TRIMESH_PROVIDER_ID)
            rec = bytearray(np.array([nf, nv, nv, nv], np.uint32).tobytes())
            rec += np.array(list(sh.bbox_min) + [0] + list(sh.bbox_max) + [0], np.float32).tobytes()
            rec += np.hstack([v, np.zeros((nv, 1))]).astype(np.float32).tobytes()
            rec += np.hstack([nrm, np.zeros((nv, 1))]).astype(np.float32).tobytes()
            rec += np.hstack([faces, np.zeros((nf, 1), np.int64)]).astype(np.uint32).tobytes()
            rec += tex.astype(np.float32).tobytes()
            self.shapes.data += rec
            if with_blas:
                boff = self.primbvh.add(16)
                self.primbvh.data += median_blas(v, faces, max_leaf)
                blas_off[s] = boff // 4
        self.leaves = bytearray()
        bmin, bmax = np.full(3, np.inf), np.full(3, -np.inf)
        for e in range(d.num_entities):
            en = d.entities[e]
            self.entities.add(0)
            rec = np.zeros(36, np.float32)
            rec[0:12] = _col_major(list(en.to_local), 3, 4)
            rec[12:24] = _col_major(list(en.to_global), 3, 4)
            rec[24:33] = _col_major(list(en.normal), 3, 3)
            rec.view(np.uint32)[33:36] = [en.shape, en.material, 0]
            self.entities.data += rec.tobytes()
            leaf = np.zeros(24, np.float32)
            leaf[0:3], leaf[4:7] = list(en.bbox_min), list(en.bbox_max)
            leaf[8:20] = _col_major(list(en.to_local), 3, 4)
            u = leaf.view(np.uint32)
            off = blas_off.get(en.shape, 0)
            u[3] = e | 0x80000000
            u[7] = en.shape
            u[20:24] = [en.flags, en.material, off & 0xFFFFFFFF, off >> 32]
            self.leaves += leaf.tobytes()
            bmin, bmax = np.minimum(bmin, list(en.bbox_min)), np.maximum(bmax, list(en.bbox_max))
        self.scene_bbox = (list(d.scene_bbox_min), list(d.scene_bbox_max))
        self.desc = d

    @staticmethod
    def _table(tbl, keep):
        buf = (C.c_uint8 * max(1, len(tbl.data))).from_buffer_copy(bytes(tbl.data) or b"\0")
        keep.append(buf)
        t = N.DbTable()
        t.data = C.cast(buf, C.c_void_p)
        t.bytes = len(tbl.data)
        t.count = tbl.count
        if tbl.lookups:
            arr = (N.LookupEntry * len(tbl.lookups))(*[N.LookupEntry(a, b, c) for a, b, c in tbl.lookups])
            keep.append(arr)
            t.lookups = C.cast(arr, C.POINTER(N.LookupEntry))
        return t

    def views(self):
        """(DatabaseView, ShadingView, keep-alive list)."""
        keep = []
        db = N.DatabaseView()
        db.entities = self._table(self.entities, keep)
        db.shapes = self._table(self.shapes, keep)
        db.trimesh_type_id, db.sphere_type_id = TRIMESH_PROVIDER_ID, SPHERE_PROVIDER_ID
        db.trimesh_primbvh = self._table(self.primbvh, keep)
        leaves = Table()
        leaves.data = self.leaves
        lt = (N.DbTable * 1)(self._table(leaves, keep))
        keep.append(lt)
        db.scene_bvh_leaves = C.cast(lt, C.POINTER(N.DbTable))
        db.num_scene_bvhs = 1
        db.scene_bbox_min[:] = self.scene_bbox[0]
        db.scene_bbox_max[:] = self.scene_bbox[1]
        d = self.desc
        sv = N.ShadingView()
        sv.film_width, sv.film_height = d.film_width, d.film_height
        sv.camera, sv.technique = d.camera, d.technique
        sv.num_materials, sv.materials = d.num_materials, d.materials
        sv.num_lights, sv.lights = d.num_lights, d.lights
        return db, sv, keep
