"""Writes the hand-written known-answer files for the asset parsers (tests/test_parser_kats.py).

The reference ships no .hdr or .obj files (.MISSING_LARGE_BLOBS), so these are written by hand from
the formats its parsers accept (RT/assets.cpp:187-400 parse_obj, :411-618 decode_radiance_color +
parse_hdr).  Every .hdr here spells its scanlines out byte by byte (run: 128 + n, value; literal:
n, then n bytes; channel-major R, G, B, E per scanline), and expected.json holds, per file, what
the reference's parse_hdr makes of it: the image (row 0 first, as Image_V3 stores it) decoded with
decode_radiance_color -- e <= 9 gives 0, else 2^(e - 136) * (m + 0.5) -- or "reject".  Which row
and column each file pixel lands in follows the resolution string: -Y puts the file's first
scanline in the LAST row (:557), -X the first pixel of a scanline in the last column (:556).

    python tests/golden/make_parser_kats.py      # rewrites tests/golden/kat/
"""
import json
import os

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat")


def decode(r, g, b, e):
    if e <= 9:
        return [0.0, 0.0, 0.0]
    mul = 2.0 ** (e - 136)
    return [mul * (r + 0.5), mul * (g + 0.5), mul * (b + 0.5)]


def scanline(w, chans):
    """chans: 4 lists of (code, bytes...) tokens, already RLE-coded by hand."""
    out = bytes([2, 2, w >> 8, w & 255])
    for ch in chans:
        for tok in ch:
            out += bytes(tok)
    return out


def expand(w, chans):
    """The per-pixel RGBE a scanline's tokens spell (file order)."""
    vals = []
    for ch in chans:
        v = []
        for tok in ch:
            if tok[0] > 128:
                v += [tok[1]] * (tok[0] & 127)
            else:
                v += list(tok[1:1 + tok[0]])
        assert len(v) == w, (len(v), w)
        vals.append(v)
    return [tuple(vals[c][x] for c in range(4)) for x in range(w)]


def image(w, h, lines, ydir, xdir):
    """Place the file's scanlines as parse_hdr does (y_advance / x_advance)."""
    img = [[None] * w for _ in range(h)]
    for k, px in enumerate(lines):
        row = k if ydir > 0 else h - 1 - k
        for i, p in enumerate(px):
            col = i if xdir > 0 else w - 1 - i
            img[row][col] = decode(*p)
    return img


# two 4-pixel scanlines: runs, literals, a run of 2 then literals, exponents 136 / 137 / 9 / 10
L0 = [[(0x84, 100)], [(4, 10, 20, 30, 40)], [(0x82, 5), (2, 6, 7)], [(0x84, 136)]]
L1 = [[(2, 1, 2), (0x82, 255)], [(0x84, 0)], [(4, 9, 8, 7, 6)], [(1, 137), (1, 9), (1, 10), (1, 136)]]


def hdr(header, res, lines):
    return header.encode() + b"\n" + res.encode() + b"\n" + b"".join(lines)


def main():
    os.makedirs(OUT, exist_ok=True)
    files, expected = {}, {}
    std = "#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n"
    px = [expand(4, L0), expand(4, L1)]
    sl = [scanline(4, L0), scanline(4, L1)]
    for name, res, yd, xd in (("minus_y_plus_x", "-Y 2 +X 4", -1, 1), ("plus_y_plus_x", "+Y 2 +X 4", 1, 1),
                              ("minus_y_minus_x", "-Y 2 -X 4", -1, -1), ("plus_y_minus_x", "+Y 2 -X 4", 1, -1)):
        files[f"{name}.hdr"] = hdr(std, res, sl)
        expected[f"{name}.hdr"] = {"w": 4, "h": 2, "image": image(4, 2, px, yd, xd)}
    # FORMAT=32-bit_rle_xyz: the reference warns and decodes the bytes as RGB
    files["xyz.hdr"] = hdr("#?RADIANCE\nFORMAT=32-bit_rle_xyz\n", "-Y 2 +X 4", sl)
    expected["xyz.hdr"] = expected["minus_y_plus_x.hdr"]
    # an unknown FORMAT defaults to RGB; PRIMARIES are parsed and unused; other lines are skipped
    files["unknown_format_primaries.hdr"] = hdr("#?RADIANCE\n# a comment\nFORMAT=32-bit_rle_foo\n"
                                                "PRIMARIES= 0.64 0.33 0.29 0.60 0.15 0.06 0.333 0.333\nEXPOSURE=1.0\n",
                                                "-Y 2 +X 4", sl)
    expected["unknown_format_primaries.hdr"] = expected["minus_y_plus_x.hdr"]
    # the resolution numbers go through strtoul(..., 0): "02" is octal 2, "0x4" hex 4
    files["octal_hex_resolution.hdr"] = hdr(std, "-Y 02 +X 0x4", sl)
    expected["octal_hex_resolution.hdr"] = expected["minus_y_plus_x.hdr"]
    # a 128-pixel scanline: a literal of exactly 128 (code 128 is a literal, not a run) and
    # runs of 127 + 1
    w = 128
    lit = list(range(128))
    L = [[(128, *lit)], [(0xFF, 3), (0x81, 4)], [(0xFF, 0), (1, 255)], [(0xFF, 140), (0x81, 130)]]
    files["literal128.hdr"] = hdr(std, f"-Y 1 +X {w}", [scanline(w, L)])
    expected["literal128.hdr"] = {"w": w, "h": 1, "image": image(w, 1, [expand(w, L)], -1, 1)}
    # rejected files
    flat = bytes([100, 10, 5, 136] * 4 + [1, 2, 9, 137] * 4)          # uncompressed scanlines
    files["flat.hdr"] = std.encode() + b"\n-Y 2 +X 4\n" + flat
    expected["flat.hdr"] = "reject"
    files["bad_scanline_length.hdr"] = hdr(std, "-Y 2 +X 4", [bytes([2, 2, 0, 5]) + sl[0][4:], sl[1]])
    expected["bad_scanline_length.hdr"] = "reject"
    files["x_major.hdr"] = hdr(std, "+X 4 -Y 2", sl)                # the reference reads +/-Y first
    expected["x_major.hdr"] = "reject"
    files["format_without_equals.hdr"] = hdr("#?RADIANCE\nFORMAT 32-bit_rle_rgbe\n", "-Y 2 +X 4", sl)
    expected["format_without_equals.hdr"] = "reject"
    files["no_resolution_newline.hdr"] = std.encode() + b"\n-Y 2 +X 4 " + b"".join(sl)
    expected["no_resolution_newline.hdr"] = "reject"
    files["zero_width.hdr"] = hdr(std, "-Y 2 +X 0", [])
    expected["zero_width.hdr"] = "reject"
    files["header_only.hdr"] = std.encode()
    expected["header_only.hdr"] = "reject"

    # OBJ (parse_obj, CounterClockwise as load_mesh passes it): expected triangles (a, b, c) in file
    # order after fan triangulation, and per-vertex normals when the faces reference any
    quad = "v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\n"
    nrm = "vn 0 0 1\nvn 0 0.6 0.8\nvn 1 0 0\nvn 0 1 0\n"
    V = [[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0]]
    N = [[0, 0, 1], [0, 0.6, 0.8], [1, 0, 0], [0, 1, 0]]
    fan = [[V[0], V[1], V[2]], [V[0], V[2], V[3]]]
    objs = {
        "v_only.obj": (quad + "f 1 2 3 4\n", fan, None),
        "v_vt.obj": (quad + "vt 0 0\nvt 1 0\nvt 1 1\nvt 0 1\nf 1/1 2/2 3/3 4/4\n", fan, None),
        "v_vn.obj": (quad + nrm + "f 1//1 2//2 3//3 4//4\n", fan, [[N[0], N[1], N[2]], [N[0], N[2], N[3]]]),
        "v_vt_vn.obj": (quad + "vt 0 0\nvt 1 0\nvt 1 1\nvt 0 1\n" + nrm + "f 1/4/4 2/3/3 3/2/2 4/1/1\n", fan,
                        [[N[3], N[2], N[1]], [N[3], N[1], N[0]]]),
        "negative_indices.obj": (quad + nrm + "f -4//-4 -3//-3 -2//-2\nf -4//1 -2//3 -1//4\n",
                                 [[V[0], V[1], V[2]], [V[0], V[2], V[3]]],
                                 [[N[0], N[1], N[2]], [N[0], N[2], N[3]]]),
        "crlf_comments_pentagon.obj": ("# comment\r\no object\r\n" + quad.replace("\n", "\r\n") + "v 0.5 1.5 0\r\n"
                                       "s off\r\nf 1 2 3 5 4\r\n",
                                       [[V[0], V[1], V[2]], [V[0], V[2], [0.5, 1.5, 0]], [V[0], [0.5, 1.5, 0], V[3]]],
                                       None),
        "two_index_face.obj": (quad + "f 1 2\n", "reject", None),
        "normals_mismatch.obj": (quad + nrm + "f 1//1 2//2 3//3\nf 1 3 4\n", "reject", None),
    }
    for name, (text, tris, normals) in objs.items():
        files[name] = text.encode()
        expected[name] = "reject" if tris == "reject" else {"triangles": tris, "normals": normals}

    for name, data in files.items():
        with open(os.path.join(OUT, name), "wb") as f:
            f.write(data)
    with open(os.path.join(OUT, "expected.json"), "w") as f:
        json.dump(expected, f, indent=1)
    print(f"wrote {len(files)} files to {OUT}")


if __name__ == "__main__":
    main()
