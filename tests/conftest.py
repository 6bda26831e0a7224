import hashlib
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "kzg-batch-verification-scheme_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long CPU test")


def load_golden(name):
    with open(os.path.join(GOLDEN, name), "rb") as f:
        data = f.read()
    with open(os.path.join(GOLDEN, "MANIFEST.json")) as f:
        manifest = json.load(f)
    assert hashlib.sha256(data).hexdigest() == manifest[name], "golden fixture %s modified" % name
    return json.loads(data)


@pytest.fixture(scope="session")
def golden():
    return load_golden
