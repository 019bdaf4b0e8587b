import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libxalm_hip.so on the device)")


def fixture_path(name):
    return os.path.join(GOLDEN, name)


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def pytest_sessionfinish(session, exitstatus):
    # XALM_ERR_LOG=path: every logits check's error (tests/bars.py), for tools/error_envelope.py
    out = os.environ.get("XALM_ERR_LOG")
    if out:
        import json

        import bars
        with open(out, "w") as f:
            json.dump(bars._LOG, f)
