"""GPU parity for the reference's four integrator switches, all 16 combinations.

The reference's UI toggles "Next Event Estimation", "Importance Sample Lights", "Importance Sample
Diffuse" and "Use Multiple Importance Sampling" (RT/raytracer.cpp:1974-1977) select separate branches
of advanced_integrator, which the GPU restates in shade_bounce (csrc/rt_kernels.hip) and the oracle in
oracle.c:
* importance_sample_lights = 0: the uniform light pick, RT/integrators.cpp:178-188;
* next_event_estimation = 0: every emissive hit counted (allow_direct_lighting), :651-657, and no
  NEE block (:738-771);
* use_mis = 0: the emissive hit after a diffuse bounce adds nothing, :658-670, and the NEE pdf
  is the light's alone, :759-763;
* importance_sample_diffuse = 0: uniform-hemisphere sampling, :780-789, and its 1 / 2 pi pdf in
  both MIS weights.
Each combination runs on the C3 and C4 presets at 192 x 108: per-sample radiance through
rt_trace_samples against the oracle's (>= 99.9 % bit-exact, the bar of test_gpu_parity.py), and
the exact-splat frame against the oracle's single-thread frame (>= 99.9 % of pixels bit-identical,
rel L2 <= 1e-6), with identical ray counts.
"""
import itertools

import numpy as np
import pytest

import oracle_binding as ob
from parity_report import REPORT
from test_gpu_parity import _sample_list, rel_l2

pytestmark = pytest.mark.gpu

SWITCHES = ("next_event_estimation", "importance_sample_lights", "use_mis", "importance_sample_diffuse")
COMBOS = list(itertools.product((0, 1), repeat=4))


@pytest.fixture(scope="module", params=["c3", "c4"])
def preset(rt, request):
    w, h = 192, 108
    scene, cam, st, fc, post = rt.load_preset(request.param, w, h)
    dev = rt.DeviceScene(scene, 0)
    yield request.param, rt, scene, cam, st, fc, dev, w, h
    dev.close()


@pytest.mark.parametrize("combo", COMBOS, ids=lambda c: "nee{}_isl{}_mis{}_isd{}".format(*c))
def test_integrator_switches(preset, combo):
    name, rt, scene, cam, st, fc, dev, w, h = preset
    st = type(st).from_buffer_copy(st)
    for k, v in zip(SWITCHES, combo):
        setattr(st, k, v)
    st.samples_per_pixel = 16
    rng = np.random.default_rng(23)
    xy, s = _sample_list(rng, w, h, 20000, st.samples_per_pixel)
    gpu, gs = dev.trace_samples(cam, st, w, h, xy, s)
    with dev.configured(splat_mode=rt.abi.RT_SPLAT_EXACT):
        frame, fs = dev.render(cam, st, fc, w, h)
    cpu, cs = ob.trace_samples(scene.desc(), cam, st, w, h, xy, s)
    cframe, cfs = ob.render(scene.desc(), cam, st, fc, w, h, rng_mode=0, threads=1)
    same = float(np.all((gpu == cpu) | (np.isnan(gpu) & np.isnan(cpu)), axis=1).mean())
    px = float(np.all(frame == cframe, axis=2).mean())
    REPORT[f"switches_{name}_" + "".join(map(str, combo))] = {
        "bit_exact_fraction": same, "frame_pixels_identical": px, "frame_rel_l2": rel_l2(frame, cframe),
        "rays": [int(fs.closest_hit_rays), int(fs.shadow_rays)], "oracle_rays": [int(cfs.closest_hit_rays),
                                                                                  int(cfs.shadow_rays)]}
    assert same >= 0.999
    assert (gs.closest_hit_rays, gs.shadow_rays) == (cs.closest_hit_rays, cs.shadow_rays)
    assert (fs.closest_hit_rays, fs.shadow_rays) == (cfs.closest_hit_rays, cfs.shadow_rays)
    if not combo[0]:
        assert fs.shadow_rays == 0                     # no NEE: no shadow ray at all
    assert px >= 0.999
    assert rel_l2(frame, cframe) <= 1e-6
    assert np.isfinite(frame).all()
