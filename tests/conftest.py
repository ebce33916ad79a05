import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def fingerprints():
    p = os.path.join(GOLDEN, "fingerprints_2p32.json")
    if not os.path.exists(p):
        pytest.skip("fingerprints_2p32.json not generated")
    with open(p) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def templates(golden):
    return {t["name"]: t for t in golden["templates"]}
