#!/usr/bin/env python3
"""Extract the reference's sampler tables into raw u8 data files.

The reference renderer's samplers read three table sets:

* ``g_strata_permutation_sets[256][64]`` (RT/samplers.cpp:140-397): per-row
  permutations of the 8x8 strata used by the stratified sampler.
* The Heitz et al. 2019 blue-noise sampler tables for 256 spp
  (RT/blue_noise_samplers/samplerBlueNoiseErrorDistribution_128x128_
  OptimizedFor_2d2d2d2d_256spp.cpp:2,7,12): ``sobol_256spp_256d[65536]``,
  ``scramblingTile[131072]``, ``rankingTile[131072]``; every value is < 256.

Only the numeric literals are read (the table *data*); no reference code is
reproduced.  Output (committed under data/):

* ``data/strata_permutation_sets.u8``  16384 bytes, row-major [256][64]
* ``data/bluenoise_256spp.u8``         327680 bytes = sobol | scrambling | ranking

Run from the repo root:  python tools/extract_tables.py [/root/reference]
"""
import hashlib
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "data")


def ints_between(text, start_pat, count):
    m = re.search(start_pat, text)
    if not m:
        raise SystemExit(f"pattern not found: {start_pat}")
    body = text[m.end():]
    end = body.index("};")
    vals = [int(v) for v in re.findall(r"-?\d+", body[:end])]
    if len(vals) != count:
        raise SystemExit(f"{start_pat}: expected {count} values, got {len(vals)}")
    if min(vals) < 0 or max(vals) > 255:
        raise SystemExit(f"{start_pat}: values outside u8 range")
    return bytes(vals)


def main():
    with open(os.path.join(REF, "Raytracer", "samplers.cpp")) as f:
        samplers = f.read()
    strata = ints_between(samplers, r"g_strata_permutation_sets\[256\]\[g_strata_count\]\s*=\s*\{", 256 * 64)
    bn_path = os.path.join(REF, "Raytracer", "blue_noise_samplers",
                           "samplerBlueNoiseErrorDistribution_128x128_OptimizedFor_2d2d2d2d_256spp.cpp")
    with open(bn_path) as f:
        bn = f.read()
    sobol = ints_between(bn, r"sobol_256spp_256d\[256\*256\]\s*=\s*\{", 65536)
    scr = ints_between(bn, r"scramblingTile\[128\*128\*8\]\s*=\s*\{", 131072)
    rank = ints_between(bn, r"rankingTile\[128\*128\*8\]\s*=\s*\{", 131072)
    os.makedirs(OUT, exist_ok=True)
    outs = {
        "strata_permutation_sets.u8": strata,
        "bluenoise_256spp.u8": sobol + scr + rank,
    }
    for name, blob in outs.items():
        with open(os.path.join(OUT, name), "wb") as f:
            f.write(blob)
        print(name, len(blob), hashlib.sha256(blob).hexdigest())


if __name__ == "__main__":
    main()
