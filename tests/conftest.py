import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) -- parity tests of the HIP path")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def index_cache(tmp_path_factory):
    from tests.common import IndexCache
    return IndexCache(str(tmp_path_factory.mktemp("svg_index")))


@pytest.fixture
def svgopt():
    """Implementation options of the library (svg_set_option; none changes a record), restored
    after the test: opt.set("host_sub", 7001), opt.reset("host_sub")."""
    import subread_amd as sa
    saved = {}

    class Opts:
        def set(self, name, value):
            if name not in saved:
                saved[name] = sa.get_option(name)
            sa.set_option(name, value)

        def reset(self, name):
            if name in saved:
                sa.set_option(name, saved[name])

    yield Opts()
    for k, v in saved.items():
        sa.set_option(k, v)
