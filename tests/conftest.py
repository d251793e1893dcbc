import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "opentelemetry-demo_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden", "spanmetrics_kat.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: full-size parity (BASELINE config sizes)")


def _ensure_built():
    if not os.path.exists(os.path.join(ROOT, "oracle", "build", "liboracle.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                       stdout=subprocess.DEVNULL)
    if not os.path.exists(os.path.join(PKG, "spanagg", "libspanagg.so")):
        subprocess.run(["make", "-C", PKG, "-j4"], check=True, stdout=subprocess.DEVNULL)
    node_addon = os.path.join(ROOT, "host", "node", "build", "spanagg.node")
    if not os.path.exists(node_addon) and os.path.exists("/usr/include/node/node_api.h"):
        subprocess.run(["make", "-C", os.path.join(ROOT, "host", "node")], check=True,
                       stdout=subprocess.DEVNULL)


_ensure_built()


@pytest.fixture(scope="session")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
