"""Independent pure-Python restatement of the reference RNG and samplers
(RT/samplers.h:3-108, RT/samplers.cpp:18-138) — used to cross-check the C
oracle and to make the golden vectors.  Small inputs only."""
import struct

import numpy as np

M32 = 0xFFFFFFFF
DATA = __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))), "data")


def wang_hash(key):
    key = (key + (~(key << 15) & M32)) & M32
    key ^= key >> 10
    key = (key + (key << 3)) & M32
    key ^= key >> 6
    key = (key + (~(key << 11) & M32)) & M32
    key ^= key >> 16
    return key


def hash3(x, y, z):
    return ((x * 73856093) ^ (y * 83492791) ^ (z * 871603259)) & M32


def hash2(x, y):
    qx = (1103515245 * ((x >> 1) ^ y)) & M32
    qy = (1103515245 * ((y >> 1) ^ x)) & M32
    return (1103515245 * (qx ^ (qy >> 3))) & M32


def xorshift(r):
    r ^= (r << 13) & M32
    r ^= r >> 17
    r ^= (r << 5) & M32
    return r


class RandomSeries:
    def __init__(self, seed):
        if seed == 0:
            seed = 0xFFFFFFFF
        h = wang_hash(seed)
        self.e = [h, h, h, h]
        a = self.next_set()
        b = self.next_set()
        c = self.next_set()
        self.next_set()
        self.e[0] = wang_hash(a[0])
        self.e[1] = wang_hash(b[1])
        self.e[2] = wang_hash(c[2])

    def next_set(self):
        self.e = [xorshift(v) for v in self.e]
        return list(self.e)

    def unilaterals(self):
        out = []
        for v in self.next_set():
            bits = (127 << 23) | (v >> 9)
            f = struct.unpack("<f", struct.pack("<I", bits))[0]
            out.append(float(np.float32(f) - np.float32(1.0)))
        return out


def sample_seed(total_frame_index, frame_count, tile, pixel_id, canonical):
    tile_seed = hash3(total_frame_index, frame_count, tile)
    inner = wang_hash(((pixel_id * 0x9E3779B9) & M32) ^ wang_hash((canonical + 0x68E31DA4) & M32))
    return wang_hash(tile_seed ^ inner)


_strata = None
_bn = None


def tables():
    global _strata, _bn
    if _strata is None:
        _strata = np.fromfile(f"{DATA}/strata_permutation_sets.u8", np.uint8).reshape(256, 64)
        _bn = np.fromfile(f"{DATA}/bluenoise_256spp.u8", np.uint8)
    return _strata, _bn


def blue_noise(x, y, index, dim):
    _, bn = tables()
    sobol, scr, rank = bn[:65536], bn[65536:65536 + 131072], bn[65536 + 131072:]
    x &= 127
    y &= 127
    index &= 255
    dim &= 255
    ranked = index ^ int(rank[dim + (x + y * 128) * 8])
    value = int(sobol[dim + ranked * 256]) ^ int(scr[(dim % 8) + (x + y * 128) * 8])
    return float(np.float32(value) / np.float32(256.0))


def f32(x):
    return np.float32(x)


def sample_2d(entropy, strategy, x, y, index, dim, bounce):
    if strategy == 1 and index > 256:
        strategy = 2
    if strategy == 1 and dim >= 4:
        strategy = 2
    u = entropy.unilaterals()
    if bounce == 0 and strategy == 1:
        return (float(f32(f32(1 / 256) * f32(u[0])) + f32(blue_noise(x, y, index, 2 * dim))),
                float(f32(f32(1 / 256) * f32(u[1])) + f32(blue_noise(x, y, index, 2 * dim + 1))))
    if bounce == 0 and strategy == 2:
        strata, _ = tables()
        off = ((73856093 * dim) & M32) ^ hash2(x, y)
        si = int(strata[off & 255, index % 64])
        sx = f32(si % 8) * f32(0.125)
        sy = f32(si // 8) * f32(0.125)
        return float(sx + f32(u[0]) * f32(0.125)), float(sy + f32(u[1]) * f32(0.125))
    return u[0], u[1]


def sample_1d(entropy, strategy, x, y, index, dim, bounce):
    if strategy == 1 and index > 256:
        strategy = 2
    if strategy == 1 and dim >= 4:
        strategy = 2
    u = entropy.unilaterals()
    if bounce == 0 and strategy == 1:
        return float(f32(f32(1 / 256) * f32(u[0])) + f32(blue_noise(x, y, index, 2 * dim)))
    if bounce == 0 and strategy == 2:
        strata, _ = tables()
        off = ((73856093 * dim) & M32) ^ hash2(x, y)
        si = int(strata[off & 255, index % 64])
        return float(f32(si) * f32(1 / 64) + f32(u[0]) * f32(1 / 64))
    return u[0]
