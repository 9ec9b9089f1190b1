"""The C ABI from a compiled C host (tests/c_host/c_host.c, linked to librt_mi355x.so the way
INTEGRATION.md §1 says): the boundary is usable without Python or ctypes.

CPU: the host links, loads the library and reports RT_ERROR_NO_DEVICE (5) when no MI355X is
visible -- the product path has no CPU fallback.  GPU: its frame (rt_render, exact splat)
equals the oracle's single-threaded frame bit for bit, and its picture (rt_render_picture +
write_bitmap) equals the oracle's output pass of that frame with the dither of frame 1.
"""
import os
import subprocess

import numpy as np
import pytest

import oracle_binding as ob

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "c_host", "c_host")


def _exe():
    if not os.path.exists(EXE):
        raise RuntimeError(f"{EXE} missing: run __graft_entry__.build() (make -C tests/c_host)")
    return EXE


def test_c_host_links_and_refuses_without_device(rt, tmp_path):
    if rt.device_count() > 0:
        pytest.skip("a GPU is visible: covered by test_c_host_frame_and_picture")
    r = subprocess.run([_exe(), "64", "64", str(tmp_path / "out.bin")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 5, (r.returncode, r.stderr)          # RT_ERROR_NO_DEVICE


@pytest.mark.gpu
def test_c_host_frame_and_picture(rt, tmp_path):
    w = h = 128
    out, bmp = tmp_path / "out.bin", tmp_path / "pic.bmp"
    r = subprocess.run([_exe(), str(w), str(h), str(out), str(bmp)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    raw = out.read_bytes()
    acc = np.frombuffer(raw, np.float32, count=w * h * 4).reshape(h, w, 4)
    pic = np.frombuffer(raw, np.uint32, count=w * h, offset=16 * w * h).reshape(h, w)
    rays = np.frombuffer(raw, np.uint64, count=2, offset=20 * w * h)
    trav = np.frombuffer(raw, np.uint64, count=4, offset=20 * w * h + 16)
    scene, cam, st, fc, post = rt.load_preset("c1", w, h)
    cpu, cs = ob.render(scene.desc(), cam, st, fc, w, h, rng_mode=0, threads=1)
    assert (int(rays[0]), int(rays[1])) == (cs.closest_hit_rays, cs.shadow_rays)
    # TraversalStats through the C ABI: C1 has no mesh, so both walks count nothing
    assert trav.tolist() == [0, 0, 0, 0] == list(cs.traversal_total().values())
    assert np.array_equal(acc, cpu)
    ref_pic = ob.postprocess(cpu, post, total_frame_index=1)
    assert np.array_equal(pic, ref_pic)
    assert np.array_equal(rt.read_bitmap(bmp, w, h), ref_pic)
