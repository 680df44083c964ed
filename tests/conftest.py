import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden():
    import json
    d = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(d, "vectors.json")) as f:
        vec = json.load(f)
    with open(os.path.join(d, "kats.json")) as f:
        kats = json.load(f)
    with open(os.path.join(d, "gf256_tables.json")) as f:
        tables = json.load(f)
    return {"vectors": vec, "kats": kats, "tables": tables}


@pytest.fixture(scope="session")
def gpu_ctx():
    """A device context on GPU 0.  Fails loudly (no skip) when the HIP library
    or device is missing: -m gpu runs only on the MI355X box."""
    import kodr_amd.device as dev
    return dev.default_context(0)
