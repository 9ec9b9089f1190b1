"""bench.py's contract pieces that need no GPU: the constants the JSON line is built
from and the measured table it reads (profiles/traffic.json from the rocprofv3 --pmc passes)
has the shape bench.py expects, so a round-end bench run on a fresh box cannot lose its
roofline block.  (The traversal figure's step counts come from the timed frames
themselves: rt_stats::trace_steps.)"""
import importlib.util
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)            # module level only: main() is behind __main__
    return mod


def test_stage_tables_agree(bench):
    assert set(bench.BYTES_PER_UNIT) <= set(bench.STAGES)
    assert set(bench.KERNEL) >= set(bench.BYTES_PER_UNIT)
    assert bench.BYTES_PER_UNIT["shade"] == 192
    assert bench.HBM_PEAK_GBS == 8000.0 and bench.L2_PEAK_GBS > bench.HBM_PEAK_GBS
    assert "c3" in bench.CONFIGS


def test_traffic_table(bench):
    """profiles/traffic.json (tools/pmc_summary.py --traffic) holds, for C3 and C4, every kernel of the
    frame the bench times (the trace launches under their phase names, DESIGN.md section 6: C3's timed frames
    merge the shadow rays into the trace launch, k_trace; C4's trace them separately, k_trace_ext /
    k_trace_shadow) and the frame's units, which bench.py's per-frame normalization (pmc_figures) needs."""
    kernels = {"c3": ("k_generate", "k_shade", "k_trace"), "c4": ("k_generate", "k_shade", "k_trace_ext", "k_trace_shadow")}
    for cfg in ("c3", "c4"):
        tj = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))["configs"][cfg]
        assert tj["frames_per_pass"] >= 1
        for k in kernels[cfg]:
            ent = tj["kernels"][k]
            assert ent["hbm_bytes_per_launch"] > 0 and ent["isolated_mean_us"] > 0
            assert ent["dispatches"] >= 1
        upf = tj["units_per_frame"]
        assert upf["k_shade"] > 0 and upf[kernels[cfg][2]] > 0


def test_host_cores(bench):
    """The CPU baseline's thread count is the cores this process may use: the affinity mask capped
    by the cgroup CPU quota, never more than os.cpu_count()."""
    hc = bench.host_cores()
    assert 1 <= hc["cores"] <= hc["affinity"] <= hc["nproc"]
    if hc["cgroup_quota_cores"] is not None:
        assert hc["cores"] <= max(1, int(hc["cgroup_quota_cores"] + 0.5))
