"""The asset parsers against hand-written known-answer files (tests/golden/kat/, written by
tests/golden/make_parser_kats.py; the reference ships no .hdr or .obj of its own).

* RGBE .hdr (parse_hdr, RT/assets.cpp:423-618): the four resolution orientations (-Y / +Y,
  +X / -X), runs, literals (a literal of exactly 128), exponents <= 9 (black), the XYZ and unknown
  FORMAT lines (read as RGB), PRIMARIES, strtoul base-0 resolution numbers; rejected: flat
  (non-RLE) scanlines, a scanline length other than the width, an X-major resolution string,
  FORMAT without '=', no newline after the resolution, a zero width, a header with no end.
* OBJ (parse_obj, RT/assets.cpp:187-400, CounterClockwise as load_mesh passes it): v, v/vt,
  v//vn, v/vt/vn faces, negative (relative) indices, CRLF lines, comments and unknown commands,
  fan triangulation of a pentagon; rejected: a two-index face, normals on only some faces.
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

KAT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kat")
EXPECTED = json.load(open(os.path.join(KAT, "expected.json")))


@pytest.mark.parametrize("name", sorted(k for k in EXPECTED if k.endswith(".hdr")))
def test_hdr_kat(rt, name):
    s = rt.Scene()
    exp = EXPECTED[name]
    if exp == "reject":
        with pytest.raises(ValueError):
            s.load_environment_map(os.path.join(KAT, name))
        assert s.desc().skydome_w == 0                     # a failed parse leaves no map
        return
    s.load_environment_map(os.path.join(KAT, name))
    d = s.desc()
    assert (d.skydome_w, d.skydome_h) == (exp["w"], exp["h"])
    got = np.ctypeslib.as_array(C.cast(d.skydome, C.POINTER(C.c_float)), shape=(exp["h"], exp["w"], 3))
    assert np.array_equal(got, np.array(exp["image"], np.float32))


def _mesh(desc, mid):
    m = desc.meshes[mid]
    n = m.triangle_count
    tris = np.ctypeslib.as_array(C.cast(m.triangles, C.POINTER(C.c_float)), shape=(n, 3, 3))
    idx = np.ctypeslib.as_array(m.indices, shape=(n,))
    orig = np.empty_like(tris)
    orig[idx] = tris                                    # BVH slot -> the file's triangle order
    nrm = None
    if m.has_normals:
        nrm = np.ctypeslib.as_array(C.cast(m.normals, C.POINTER(C.c_float)), shape=(n, 3, 3)).copy()
    return orig, nrm


@pytest.mark.parametrize("name", sorted(k for k in EXPECTED if k.endswith(".obj")))
def test_obj_kat(rt, name):
    s = rt.Scene()
    exp = EXPECTED[name]
    if exp == "reject":
        with pytest.raises(ValueError):
            s.load_obj_mesh(os.path.join(KAT, name))
        return
    mid = s.load_obj_mesh(os.path.join(KAT, name))
    tris, nrm = _mesh(s.desc(), mid)
    assert np.array_equal(tris, np.array(exp["triangles"], np.float32))
    if exp["normals"] is None:
        assert nrm is None
    else:
        assert np.array_equal(nrm, np.array(exp["normals"], np.float32))
