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


def _stale(target, *src_dirs):
    """True when `target` is missing or older than any source file under
    src_dirs (a stale in-tree library must never be tested silently)."""
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    for d in src_dirs:
        for base, _, files in os.walk(d):
            for f in files:
                if f.endswith((".hip", ".cpp", ".cc", ".c", ".h")) and os.path.getmtime(os.path.join(base, f)) > t:
                    return True
    return False


def _ensure_built():
    if _stale(os.path.join(ROOT, "oracle", "build", "liboracle.so"), os.path.join(ROOT, "oracle")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                       stdout=subprocess.DEVNULL)
    if _stale(os.path.join(PKG, "spanagg", "libspanagg.so"), os.path.join(PKG, "csrc"), os.path.join(ROOT, "include")):
        # make's own rules would rebuild every object (build/*.o never travel
        # to the GPU box), so the staleness test above decides; then a full build
        subprocess.run(["make", "-C", PKG, "-j8"], check=True, stdout=subprocess.DEVNULL)
    node_addon = os.path.join(ROOT, "host", "node", "build", "spanagg.node")
    if _stale(node_addon, os.path.join(ROOT, "host", "node", "binding"), os.path.join(ROOT, "include")) and \
            os.path.exists("/usr/include/node/node_api.h"):
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
