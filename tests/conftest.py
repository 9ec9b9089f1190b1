"""Shared test setup.

* registers the `gpu` marker (tests that need a real MI355X);
* imports the product package `buas-pathtracer_amd/` as `buas_pathtracer_amd`;
* exposes the CPU oracle (test infrastructure, oracle/liboracle.so).
"""
import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def _import_package():
    name = "buas_pathtracer_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(
        name, os.path.join(ROOT, "buas-pathtracer_amd", "__init__.py"),
        submodule_search_locations=[os.path.join(ROOT, "buas-pathtracer_amd")])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    _import_package()


@pytest.fixture(scope="session")
def rt():
    return _import_package()


@pytest.fixture(scope="session")
def oracle():
    import oracle_binding
    return oracle_binding.load()


@pytest.fixture(scope="session", autouse=True)
def _parity_report():
    """Write the GPU tests' measured parity figures to gpurun_out/parity_report.json."""
    yield
    from parity_report import REPORT
    if not REPORT:
        return
    import json
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "parity_report.json"), "w") as f:
        json.dump(REPORT, f, indent=1)
