"""The reference-side binding in integration/ compiles against the reference's own headers (the drop-in proof:
it implements srsran::ldpc_decoder / ldpc_decoder_factory over the srsgpu C ABI). Compile-only; needs /root/reference."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "include", "srsran")), reason="reference tree absent")
@pytest.mark.parametrize("src", ["ldpc_decoder_gpu.cpp", "hw_accelerator_pusch_dec_gpu.cpp",
                                 "hw_accelerator_pdsch_enc_gpu.cpp", "pusch_chain_gpu.cpp", "pdsch_chain_gpu.cpp",
                                 "ofdm_gpu.cpp", "upper_phy_factories_gpu.cpp"])
def test_binding_compiles_against_reference_headers(src, tmp_path):
    cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-fsyntax-only", "-DFMT_HEADER_ONLY",
           f"-I{REF}/include", f"-I{REF}", f"-I{REF}/external/fmt/include", f"-I{REF}/external", f"-I{ROOT}/include",
           f"-I{ROOT}/integration", "-I/opt/rocm/include", "-x", "c++", "-D__HIP_PLATFORM_AMD__", os.path.join(ROOT, "integration", src)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libsrshal.so")),
                    reason="HAL harness not built (oracle/build_hal.sh)")
def test_hal_harness_links_reference_processors_with_gpu_bindings():
    """oracle/build_hal.sh links the reference's pusch_decoder_hw_impl / pdsch_encoder_hw_impl / pusch_decoder_impl /
    pdsch_encoder_impl with the integration/ bindings (-Wl,--no-undefined): the library loads and exports the harness
    entry points (no GPU call here; the GPU run is tests/test_hal_gpu.py)."""
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libsrshal.so"))
    for sym in ("hal_create", "hal_destroy", "hal_pusch_decode", "hal_pdsch_encode", "hal_pool_create",
                "hal_pool_decode", "hal_pool_destroy"):
        assert hasattr(lib, sym)


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libsrschain.so")),
                    reason="chain harness not built (oracle/build_chain.sh)")
def test_chain_harness_links_reference_processors_with_gpu_signal_chain():
    """oracle/build_chain.sh links the reference's pusch_processor_impl / pdsch_processor_impl (with the reference's
    UCI decoder, UL-SCH demultiplexer, PT-RS generator) with the signal-chain bindings (-Wl,--no-undefined): the
    library loads and exports the harness entry points (the GPU run is tests/test_chain_gpu.py)."""
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libsrschain.so"))
    for sym in ("chain_create", "chain_destroy", "chain_ue_tx", "chain_pusch_process", "chain_pdsch_process",
                "chain_ofdm_modulate", "chain_ofdm_demodulate", "chain_factory_validate", "chain_ul_create",
                "chain_dl_create"):
        assert hasattr(lib, sym)
