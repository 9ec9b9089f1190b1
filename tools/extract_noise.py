#!/usr/bin/env python3
"""Extract the reference's dither noise textures into a raw u8 data file.

The reference's output pass (RT/raytracer.cpp:2103-2171) dithers with
``g_blue_noise3[total_frame_index % 8]``, loaded from
``data/noise/LDR_RGB1_{0..7}.png`` (RT/assets.cpp:63-113) as R8G8B8: the first
three channels of each RGBA pixel (RT/assets.cpp:22-45).

The PNGs are image data.  They are decoded here by a small PNG reader (zlib +
the five PNG row filters, 8-bit RGBA only), so no reference code or external
image loader runs.  Output (committed under data/):

* ``data/dither_rgb1_256.u8``  8 x 256 x 256 x 3 bytes = 1572864, texture-major, row-major, RGB

Run from the repo root:  python tools/extract_noise.py [/root/reference]
"""
import hashlib
import os
import struct
import sys
import zlib

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "data", "dither_rgb1_256.u8")


def paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    if pa <= pb and pa <= pc:
        return a
    return b if pb <= pc else c


def decode_rgba8(path):
    data = open(path, "rb").read()
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        raise SystemExit(f"{path}: not a PNG")
    i, idat, hdr = 8, b"", None
    while i < len(data):
        n = struct.unpack(">I", data[i:i + 4])[0]
        kind, body = data[i + 4:i + 8], data[i + 8:i + 8 + n]
        if kind == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif kind == b"IDAT":
            idat += body
        i += 12 + n
    w, h, depth, ctype, _, _, interlace = hdr
    if depth != 8 or ctype != 6 or interlace != 0:
        raise SystemExit(f"{path}: only 8-bit non-interlaced RGBA is handled")
    raw = zlib.decompress(idat)
    bpp, stride = 4, 4 * w
    out = bytearray(h * stride)
    prev = bytearray(stride)
    pos = 0
    for y in range(h):
        f = raw[pos]
        line = bytearray(raw[pos + 1:pos + 1 + stride])
        pos += 1 + stride
        for x in range(stride):
            a = line[x - bpp] if x >= bpp else 0
            b = prev[x]
            c = prev[x - bpp] if x >= bpp else 0
            if f == 1:
                line[x] = (line[x] + a) & 255
            elif f == 2:
                line[x] = (line[x] + b) & 255
            elif f == 3:
                line[x] = (line[x] + ((a + b) >> 1)) & 255
            elif f == 4:
                line[x] = (line[x] + paeth(a, b, c)) & 255
            elif f != 0:
                raise SystemExit(f"{path}: bad filter {f}")
        out[y * stride:(y + 1) * stride] = line
        prev = line
    return w, h, bytes(out)


def main():
    blob = bytearray()
    for k in range(8):
        w, h, rgba = decode_rgba8(os.path.join(REF, "Raytracer", "data", "noise", f"LDR_RGB1_{k}.png"))
        if (w, h) != (256, 256):
            raise SystemExit("unexpected texture size")
        for p in range(w * h):
            blob += rgba[4 * p:4 * p + 3]
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "wb") as f:
        f.write(blob)
    print(OUT, len(blob), hashlib.sha256(blob).hexdigest())


if __name__ == "__main__":
    main()
