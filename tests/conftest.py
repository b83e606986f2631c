import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libdcf_hip.so on cuda:0)")
    config.addinivalue_line("markers", "config: full-size BASELINE.json config parity (run last)")


def pytest_collection_modifyitems(session, config, items):
    """Full-size config tests run after everything else, so `-x` still reports the
    smaller tests first (stable order otherwise)."""
    items.sort(key=lambda it: it.get_closest_marker("config") is not None)


def load_golden(name):
    with open(os.path.join(GOLDEN, f"{name}.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def hip_lib():
    """The product library, built in-tree; compute tests must not run without it.  An explicit
    DCF_HIP_LIB (a diagnostic or A/B build) is loaded as it is, without rebuilding the default."""
    from dcf_amd import build
    if not os.environ.get("DCF_HIP_LIB"):
        build.build()
    import dcf_amd
    return dcf_amd.load()
