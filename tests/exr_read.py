"""Test-side reader for the uncompressed float OpenEXR files igx writes
(independent of the writer: parses the header attributes and the offset table)."""
import struct

import numpy as np


def read_exr(path):
    data = open(path, "rb").read()
    magic, version = struct.unpack_from("<II", data, 0)
    assert magic == 20000630 and (version & 0xFF) == 2, (magic, version)
    pos = 8
    attrs = {}
    while data[pos] != 0:
        end = data.index(b"\0", pos)
        name = data[pos:end].decode()
        pos = end + 1
        end = data.index(b"\0", pos)
        typ = data[pos:end].decode()
        pos = end + 1
        (size,) = struct.unpack_from("<i", data, pos)
        pos += 4
        attrs[name] = (typ, data[pos:pos + size])
        pos += size
    pos += 1
    chans = []
    raw = attrs["channels"][1]
    p = 0
    while raw[p] != 0:
        end = raw.index(b"\0", p)
        nm = raw[p:end].decode()
        ptype = struct.unpack_from("<i", raw, end + 1)[0]
        chans.append((nm, ptype))
        p = end + 1 + 16
    assert attrs["compression"][1] == b"\0", "only NO_COMPRESSION"
    x0, y0, x1, y1 = struct.unpack("<4i", attrs["dataWindow"][1])
    w, h = x1 - x0 + 1, y1 - y0 + 1
    offsets = struct.unpack_from(f"<{h}Q", data, pos)
    img = {nm: np.zeros((h, w), np.float32) for nm, _ in chans}
    for off in offsets:
        y, nbytes = struct.unpack_from("<ii", data, off)
        line = np.frombuffer(data, np.float32, count=nbytes // 4, offset=off + 8).reshape(len(chans), w)
        for k, (nm, ptype) in enumerate(chans):
            assert ptype == 2  # FLOAT
            img[nm][y - y0] = line[k]
    return img, attrs
