import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    # torch ships its own HIP runtime: it must initialise the device before libuno_kkt.so's runtime does,
    # or it reports no GPU (tests that hand torch device buffers to the library rely on it)
    try:
        import torch
        torch.cuda.is_available()
    except Exception:  # noqa: BLE001 -- torch is plumbing for a few tests only
        pass
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: full-size (C3) parity properties")
    config.addinivalue_line("markers", "needs_driver: runs the reference Uno core through oracle/_ref/uno_kkt_driver")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the oracle and the HIP library once per session (in-tree, no JIT cache)."""
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    if not os.path.exists(os.path.join(ROOT, "uno_amd", "libuno_kkt.so")) or \
            not os.path.exists(os.path.join(ROOT, "uno_amd", "libarrowband.so")):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "uno_amd")], check=True)
