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
