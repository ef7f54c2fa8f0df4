"""CPU-side check of the drop-in boundary: the C-ABI library builds, loads and exports every function declared in
include/srsgpu_phy.h (no compute call: there is no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "srsgpu_phy.h")
LIB = os.path.join(ROOT, "srsran-5g_amd", "lib", "libsrsgpu_phy.so")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(srsgpu_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_api():
    fns = declared_functions()
    assert "srsgpu_ldpc_decode" in fns and "srsgpu_context_create" in fns


@pytest.mark.skipif(not os.path.exists(LIB), reason="libsrsgpu_phy.so not built")
def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if line.strip())
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    import torch  # noqa: F401  (share torch's HIP runtime, as the product binding does)
    lib = ctypes.CDLL(LIB)
    for f in declared_functions():
        assert hasattr(lib, f)
    assert lib.srsgpu_version() >= 100


@pytest.mark.skipif(not os.path.exists(LIB), reason="libsrsgpu_phy.so not built")
def test_python_binding_lists_header_symbols():
    import srsgpu
    assert sorted(srsgpu.EXPORTED_SYMBOLS) == declared_functions()


@pytest.mark.skipif(not os.path.exists(LIB), reason="libsrsgpu_phy.so not built")
def test_no_device_fails_loudly():
    import torch
    import srsgpu
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(srsgpu.SrsGpuError):
        srsgpu.Context(0)
