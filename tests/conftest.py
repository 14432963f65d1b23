import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
DATA = os.path.join(REPO, "tests", "data")
TUTORIAL = os.path.join(DATA, "tutorial.fil")
GOLDEN_XML = os.path.join(DATA, "golden_overview.xml")
GOLDEN_CANDS = os.path.join(DATA, "golden_candidates.peasoup")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no HIP device visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def C():
    import peasoup_amd

    return peasoup_amd._C


@pytest.fixture(scope="session")
def golden():
    from peasoup_amd.utils.outputs import OverviewFile

    return OverviewFile(GOLDEN_XML)
