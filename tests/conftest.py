"""Shared test setup: paths, builds, the `gpu` marker."""
import os
import subprocess
import sys

import pytest

try:  # torch first: it and libtiresias_fp.so must share one HIP runtime (same SONAME)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is plumbing for the device-path tests only
    torch = None

# The library reads its test knobs (TFP_GENERIC, TFP_WIDE_POINTS, TFP_INDEX_FULL, ...; tfp::knob)
# only under TFP_TEST_KNOBS: set for the whole session, so a test's monkeypatched knob reaches the
# engines it creates, while a production process's environment never selects a kernel.
os.environ["TFP_TEST_KNOBS"] = "1"

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "asterisk-tiresias_amd")
for p in (PKG, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) — run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running check")


def _make(path):
    subprocess.run(["make", "-s", "-C", path], check=True)


@pytest.fixture(scope="session")
def oracle():
    _make(os.path.join(REPO, "oracle"))
    import oracle_py
    return oracle_py


@pytest.fixture(scope="session")
def tfp_lib():
    # make's dependency check: a library older than any of its sources or headers is rebuilt
    # from the tree under test (a shipped .so is reused only when it is the current build)
    _make(PKG)
    import tiresias_amd
    return tiresias_amd


@pytest.fixture(scope="session")
def engine(tfp_lib):
    if tfp_lib.device_count() < 1:
        pytest.skip("no GPU visible")
    e = tfp_lib.Engine(0)
    yield e
    e.close()
