"""The C-ABI library loads and exports every function declared in include/*.h;
without a GPU the product refuses to run (no CPU fallback)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in ("rt_abi.h", "rt_host.h"):
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(rth?_\w+)\s*\(", text, flags=re.M):
            names.add(m.group(1))
    return sorted(names)


def test_every_declared_symbol_is_exported(rt):
    lib = rt.lib()
    names = declared_functions()
    assert len(names) > 40
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.rt_abi_version() == 8


def test_ctypes_table_covers_header(rt):
    from buas_pathtracer_amd.abi import ABI_FUNCTIONS, HOST_FUNCTIONS
    assert set(declared_functions()) == set(ABI_FUNCTIONS) | set(HOST_FUNCTIONS)


def test_struct_sizes_match_reference_layout(rt):
    import ctypes as C
    a = rt.abi
    assert C.sizeof(a.Material) == 68                  # RT/scene.h:15-29
    assert C.sizeof(a.BvhNode) == 32                   # RT/bvh.h:31-37
    assert C.sizeof(a.M4x4Inv) == 128
    assert C.sizeof(a.FilterCache) == 8 + 512 * 4     # RT/Raytracer.h:34-40


def test_stats_layout_matches_header(rt, tmp_path):
    """The ctypes rt_stats (the TraversalStats fields of ABI v6, the reference-unit ones of v7) has the
    C header's layout."""
    import ctypes as C
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("needs gcc")
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "rt_abi.h"\n'
                   'int main(void) { printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(rt_stats), offsetof(rt_stats, traversal), '
                   'offsetof(rt_stats, trace_steps), sizeof(rt_traversal_stats), offsetof(rt_stats, traversal_ref), '
                   'offsetof(rt_scene_config, traversal_ref)); return 0; }\n')
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    size, off_trav, off_steps, tsize, off_ref, off_cfg_ref = map(int, subprocess.check_output([str(exe)]).split())
    a = rt.abi
    assert C.sizeof(a.Stats) == size
    assert a.Stats.traversal.offset == off_trav and a.Stats.trace_steps.offset == off_steps
    assert a.Stats.traversal_ref.offset == off_ref and a.SceneConfig.traversal_ref.offset == off_cfg_ref
    assert C.sizeof(a.TraversalStats) == tsize == 32


def test_no_cpu_fallback_without_gpu(rt):
    if rt.device_count() > 0:
        pytest.skip("a GPU is visible")
    scene, cam, st, fc, post = rt.load_preset("c1", 32, 32)
    with pytest.raises(rt.RenderError) as e:
        rt.DeviceScene(scene, 0)
    assert e.value.code == rt.abi.RT_ERROR_NO_DEVICE


def test_scene_config_defaults(rt):
    """rt_scene_default_config (no device needed): every per-scene setting starts at 'inherit the
    process setter' or 'auto', and the ctypes mirror has the C layout."""
    import ctypes as C
    a = rt.abi
    assert C.sizeof(a.SceneConfig) == 88
    c = a.SceneConfig()
    assert rt.lib().rt_scene_default_config(C.byref(c)) == 0
    assert (c.splat_mode, c.shard_mode, c.env_sampling) == (a.RT_CONFIG_INHERIT,) * 3
    assert (c.partitions, c.path_pool, c.fuse_paths, c.splat_chunk, c.splat_ring) == (0, 0, -1, 0, 0)
    assert c.sample_budget_gb < 0 and c.resolve_tall_pixels == 0 and c.debug_traversal == 0
    assert c.traversal_ref == 0 and c.drain_every == 0 and c.shadow_launch == a.RT_SHADOW_LAUNCH_AUTO
