import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "hd-gnn_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def pytest_sessionfinish(session, exitstatus):
    path = os.environ.get("HDG_PARITY_REPORT")
    if not path:
        return
    import json
    from tests import _errlog
    if _errlog.RECORDS:
        with open(path, "w") as f:
            json.dump(_errlog.RECORDS, f, indent=0)


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
