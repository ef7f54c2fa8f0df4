import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "srsran-5g_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # numpy restatements (test infrastructure only)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); parity tests through the C-ABI")
    config.addinivalue_line("markers", "ref: needs oracle/_ref/libsrsref.so (reference built from its own sources)")


def pytest_collection_finish(session):
    """A GPU run initialises torch's HIP runtime before any test loads a ctypes harness (oracle/_ref/libsrschain.so
    links the system HIP runtime): a harness that brings the device up first leaves torch.cuda unavailable for the
    tests that follow it in the same process."""
    if any(item.get_closest_marker("gpu") for item in session.items):
        try:
            import torch
            torch.cuda.is_available()
        except Exception:  # noqa: BLE001
            pass
