"""pytest configuration: `gpu` marker and import paths.

CPU tests (-m "not gpu") cover the oracle against the golden vectors, host
logic, the multi-rank sharding path over gloo, and that libgdist.so loads
and exports every symbol of include/gdist.h. GPU tests (-m gpu) are the
parity tests proper: the HIP path through the C-ABI against the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "genome.distance_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgdist.so on the device)")


@pytest.fixture(scope="session")
def ctx():
    import gdist
    return gdist.Context.default(0)


@pytest.fixture
def opts(ctx):
    """opts(name=value, ...) sets tuning options of the shared context
    (gdist_ctx_set_option) for one test; they are restored at teardown."""
    old = {}

    def set_(**kw):
        for k, v in kw.items():
            if k not in old:
                old[k] = ctx.option(k)
            ctx.set_option(k, v)
    yield set_
    for k, v in old.items():
        ctx.set_option(k, v)
