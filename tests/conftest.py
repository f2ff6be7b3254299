import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "llmsys-project-flashattn_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")


def pytest_collection_modifyitems(session, config, items):
    """The host-sanitizer run of the C ABI (tests/test_asan.py) goes last: it is
    infrastructure, and under ``-x`` a failure there must not stop the parity tests from
    running (GPUTEST_r05 stopped at it before any of them)."""
    items.sort(key=lambda it: it.nodeid.startswith("tests/test_asan.py") or "/test_asan.py" in it.nodeid)


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")


# ---- measured parity record ------------------------------------------------------------
# GPU parity tests call parity_record(test, case, max_abs=..., bound=...) with the error
# they measured; at session end the records go to $MT_PARITY_OUT (default
# gpurun_out/parity.json, which gpurun copies back; profiles/parity_rNN.json is the
# committed copy).
_PARITY = []


@pytest.fixture(scope="session")
def parity_record():
    def rec(test, case, **vals):
        clean = {k: (float(v) if hasattr(v, "__float__") else v) for k, v in vals.items()}
        _PARITY.append({"test": test, "case": case, **clean})
    return rec


def pytest_sessionfinish(session, exitstatus):
    if not _PARITY:
        return
    import json
    out = os.environ.get("MT_PARITY_OUT", os.path.join(ROOT, "gpurun_out", "parity.json"))
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump({"exitstatus": int(exitstatus), "records": _PARITY}, f, indent=1)
