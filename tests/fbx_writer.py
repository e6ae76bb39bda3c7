"""Test-side binary FBX writer: builds FBX 7.4 / 7.5 files from node trees so that the reader's container
and transform rules (rsd/fbx.py) are tested on inputs whose geometry is known.  Test infrastructure only."""
import struct
import zlib

import numpy as np

MAGIC = b"Kaydara FBX Binary  \x00"


class N:
    """A record: name, properties (python values or numpy arrays), children."""

    def __init__(self, name, *props, children=()):
        self.name, self.props, self.children = name, list(props), list(children)


def _prop(v, compress):
    if isinstance(v, np.ndarray):
        code, dt = {np.dtype(np.float64): (b"d", "<f8"), np.dtype(np.float32): (b"f", "<f4"),
                    np.dtype(np.int32): (b"i", "<i4"), np.dtype(np.int64): (b"l", "<i8")}[v.dtype]
        raw = np.ascontiguousarray(v, dt).tobytes()
        body = zlib.compress(raw) if compress else raw
        return code + struct.pack("<III", v.size, 1 if compress else 0, len(body)) + body
    if isinstance(v, bool):
        return b"C" + struct.pack("<?", v)
    if isinstance(v, int):
        return (b"I" + struct.pack("<i", v)) if -2**31 <= v < 2**31 else (b"L" + struct.pack("<q", v))
    if isinstance(v, float):
        return b"D" + struct.pack("<d", v)
    if isinstance(v, (bytes, str)):
        b = v.encode() if isinstance(v, str) else v
        return b"S" + struct.pack("<I", len(b)) + b
    raise TypeError(type(v))


def _record(n, offset, wide, compress):
    hdr = 25 if wide else 13
    props = b"".join(_prop(v, compress) for v in n.props)
    name = n.name.encode()
    head_len = hdr + len(name) + len(props)
    body = b""
    pos = offset + head_len
    for c in n.children:
        rb = _record(c, pos, wide, compress)
        body += rb
        pos += len(rb)
    if n.children:
        body += b"\x00" * hdr
    end = offset + head_len + len(body)
    fmt = "<QQQB" if wide else "<IIIB"
    return struct.pack(fmt, end, len(n.props), len(props), len(name)) + name + props + body


def write(nodes, version=7500, compress=True) -> bytes:
    wide = version >= 7500
    out = MAGIC + b"\x1a\x00" + struct.pack("<I", version)
    for n in nodes:
        out += _record(n, len(out), wide, compress)
    out += b"\x00" * (25 if wide else 13)
    return out


def p70(**props):
    """Properties70 with P records: name -> tuple of values (the type strings are not read)."""
    kids = []
    for k, v in props.items():
        k = k.replace("_", " ") if k.startswith("Lcl") else k
        vals = v if isinstance(v, tuple) else (v,)
        kids.append(N("P", k, "", "", "A", *vals))
    return N("Properties70", children=kids)


def mesh_geometry(gid, positions, polygons, uv=None, materials=None):
    """A Geometry "Mesh": polygons = lists of control-point indices (the last stored as ~index)."""
    pvi = []
    for poly in polygons:
        pvi += list(poly[:-1]) + [~poly[-1]]
    kids = [N("Vertices", np.asarray(positions, np.float64).reshape(-1)),
            N("PolygonVertexIndex", np.asarray(pvi, np.int32))]
    if uv is not None:
        kids.append(N("LayerElementUV", 0, children=[
            N("MappingInformationType", "ByPolygonVertex"), N("ReferenceInformationType", "Direct"),
            N("UV", np.asarray(uv, np.float64).reshape(-1))]))
    if materials is not None:
        kids.append(N("LayerElementMaterial", 0, children=[
            N("MappingInformationType", "ByPolygon"), N("ReferenceInformationType", "IndexToDirect"),
            N("Materials", np.asarray(materials, np.int32))]))
    return N("Geometry", gid, "\x00\x01Geometry", "Mesh", children=kids)


def model(mid, name, **props):
    return N("Model", mid, name + "\x00\x01Model", "Mesh", children=[p70(**props)])


def material(mid, name, **props):
    return N("Material", mid, name + "\x00\x01Material", "", children=[p70(**props)])


def scene(objects, connections, templates=None):
    """Top-level records: Definitions (optional property templates per object type), Objects, Connections."""
    defs = []
    for typ, props in (templates or {}).items():
        defs.append(N("ObjectType", typ, children=[N("PropertyTemplate", "Fbx" + typ, children=[p70(**props)])]))
    cons = [N("C", "OO", c, p) for c, p in connections]
    return [N("Definitions", children=defs), N("Objects", children=objects), N("Connections", children=cons)]
