"""The reference-side binding in integration/ compiles against the reference's own headers (the drop-in proof:
it implements srsran::ldpc_decoder / ldpc_decoder_factory over the srsgpu C ABI). Compile-only; needs /root/reference."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "include", "srsran")), reason="reference tree absent")
@pytest.mark.parametrize("src", ["ldpc_decoder_gpu.cpp"])
def test_binding_compiles_against_reference_headers(src, tmp_path):
    cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-fsyntax-only", "-DFMT_HEADER_ONLY",
           f"-I{REF}/include", f"-I{REF}/external/fmt/include", f"-I{REF}/external", f"-I{ROOT}/include",
           "-I/opt/rocm/include", "-x", "c++", "-D__HIP_PLATFORM_AMD__", os.path.join(ROOT, "integration", src)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
