"""srsgpu — Python host binding of libsrsgpu_phy.so (the MI355X 5G NR PHY kernels), over its C ABI
(include/srsgpu_phy.h).

The Python side mirrors the srsRAN interfaces it replaces (names, argument meaning and error behaviour) so the parity
tests read like the reference's own tests:

  * ``LdpcDecoder.decode(llrs, cfg)``  <->  srsran::ldpc_decoder::decode()
    (include/srsran/phy/upper/channel_coding/ldpc/ldpc_decoder.h:72)

Device memory and streams come from PyTorch (ROCm); PyTorch is plumbing only — every codeblock is processed by the
HIP kernels in libsrsgpu_phy.so. There is no CPU fallback: if the library or a HIP device is missing, the calls raise.
"""
import ctypes
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

try:  # Import torch first: it loads its own libamdhip64.so.7, which our library then shares (one HIP runtime).
    import torch
except ImportError:  # pragma: no cover - torch is part of the image
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
# SRSGPU_LIB selects another build of the library (e.g. an instrumented one under a different SRSGPU_OUT_DIR).
LIB_PATH = os.environ.get("SRSGPU_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libsrsgpu_phy.so"))

SRSGPU_OK = 0
CRC24A, CRC24B, CRC24C, CRC16, CRC11, CRC6 = range(6)
CRC_NONE = 255
IMPL_GENERIC, IMPL_SIMD = 0, 1
IMPL_BY_NAME = {"generic": IMPL_GENERIC, "avx2": IMPL_SIMD, "avx512": IMPL_SIMD, "neon": IMPL_SIMD,
                "auto": IMPL_SIMD, "simd": IMPL_SIMD}
BG_K = {1: 22, 2: 10}
BG_N_SHORT = {1: 66, 2: 50}


class SrsGpuError(RuntimeError):
    pass


class LdpcDecoderConfig(ctypes.Structure):
    """srsgpu_ldpc_decoder_config (include/srsgpu_phy.h)."""
    _fields_ = [
        ("base_graph", ctypes.c_uint8),
        ("crc_poly", ctypes.c_uint8),
        ("lifting_size", ctypes.c_uint16),
        ("nof_filler_bits", ctypes.c_uint16),
        ("nof_crc_bits", ctypes.c_uint8),
        ("max_iterations", ctypes.c_uint8),
        ("scaling_factor", ctypes.c_float),
        ("llr_offset", ctypes.c_uint32),
        ("nof_llrs", ctypes.c_uint32),
        ("out_offset", ctypes.c_uint32),
    ]


assert ctypes.sizeof(LdpcDecoderConfig) == 24


class PuschCbConfig(ctypes.Structure):
    """srsgpu_pusch_cb_config (include/srsgpu_phy.h)."""
    _fields_ = [
        ("base_graph", ctypes.c_uint8),
        ("rv", ctypes.c_uint8),
        ("modulation_order", ctypes.c_uint8),
        ("crc_poly", ctypes.c_uint8),
        ("lifting_size", ctypes.c_uint16),
        ("nof_filler_bits", ctypes.c_uint16),
        ("nof_crc_bits", ctypes.c_uint8),
        ("max_iterations", ctypes.c_uint8),
        ("new_data", ctypes.c_uint8),
        ("use_early_stop", ctypes.c_uint8),
        ("scaling_factor", ctypes.c_float),
        ("Nref", ctypes.c_uint32),
        ("rm_length", ctypes.c_uint32),
        ("llr_offset", ctypes.c_uint32),
        ("harq_offset", ctypes.c_uint32),
        ("out_offset", ctypes.c_uint32),
    ]


assert ctypes.sizeof(PuschCbConfig) == 36


class PdschTbConfig(ctypes.Structure):
    """srsgpu_pdsch_tb_config (include/srsgpu_phy.h)."""
    _fields_ = [
        ("base_graph", ctypes.c_uint8),
        ("rv", ctypes.c_uint8),
        ("modulation_order", ctypes.c_uint8),
        ("nof_layers", ctypes.c_uint8),
        ("tbs_bytes", ctypes.c_uint32),
        ("nof_ch_symbols", ctypes.c_uint32),
        ("Nref", ctypes.c_uint32),
        ("tb_offset", ctypes.c_uint32),
        ("cw_offset", ctypes.c_uint32),
    ]


assert ctypes.sizeof(PdschTbConfig) == 24


class PuschTbConfig(ctypes.Structure):
    """srsgpu_pusch_tb_config (include/srsgpu_phy.h)."""
    _fields_ = [
        ("base_graph", ctypes.c_uint8),
        ("rv", ctypes.c_uint8),
        ("modulation_order", ctypes.c_uint8),
        ("nof_layers", ctypes.c_uint8),
        ("new_data", ctypes.c_uint8),
        ("use_early_stop", ctypes.c_uint8),
        ("max_iterations", ctypes.c_uint8),
        ("reserved", ctypes.c_uint8),
        ("scaling_factor", ctypes.c_float),
        ("tbs_bytes", ctypes.c_uint32),
        ("nof_ch_symbols", ctypes.c_uint32),
        ("Nref", ctypes.c_uint32),
        ("llr_offset", ctypes.c_uint32),
        ("harq_offset", ctypes.c_uint32),
        ("cb_offset", ctypes.c_uint32),
        ("tb_offset", ctypes.c_uint32),
    ]


assert ctypes.sizeof(PuschTbConfig) == 40


class PdschModConfig(ctypes.Structure):
    """srsgpu_pdsch_mod_config (include/srsgpu_phy.h): one PDSCH transmission of pdsch_modulator::config_t."""
    _fields_ = [
        ("rnti", ctypes.c_uint16),
        ("n_id", ctypes.c_uint16),
        ("modulation_order", ctypes.c_uint8),
        ("nof_layers", ctypes.c_uint8),
        ("nof_ports", ctypes.c_uint8),
        ("start_symbol", ctypes.c_uint8),
        ("nof_symbols", ctypes.c_uint8),
        ("dmrs_type", ctypes.c_uint8),
        ("nof_cdm_groups_without_data", ctypes.c_uint8),
        ("reserved", ctypes.c_uint8),
        ("dmrs_symbol_mask", ctypes.c_uint16),
        ("bwp_start_rb", ctypes.c_uint16),
        ("bwp_size_rb", ctypes.c_uint16),
        ("rb_start", ctypes.c_uint16),
        ("nof_rb", ctypes.c_uint16),
        ("pad", ctypes.c_uint16),
        ("scaling", ctypes.c_float),
        ("precoding", ctypes.c_float * 32),
        ("cw_offset", ctypes.c_uint32),
        ("nof_bits", ctypes.c_uint32),
        ("grid_index", ctypes.c_uint32),
    ]


assert ctypes.sizeof(PdschModConfig) == 168


class RePatternC(ctypes.Structure):
    """srsgpu_re_pattern (include/srsgpu_phy.h)."""
    _fields_ = [("crb_mask", ctypes.c_void_p), ("re_mask", ctypes.c_uint16), ("symbol_mask", ctypes.c_uint16)]


class AllocExtC(ctypes.Structure):
    """srsgpu_alloc_ext (include/srsgpu_phy.h): CRB mask, reserved RE patterns and per-PRG precoding."""
    _fields_ = [("crb_mask", ctypes.c_void_p), ("reserved", ctypes.c_void_p), ("nof_reserved", ctypes.c_uint32),
                ("prg_size", ctypes.c_uint16), ("nof_prg", ctypes.c_uint16), ("prg_weights", ctypes.c_void_p)]
CB_MSG_STRIDE = 1056


class PdschDmrsConfig(ctypes.Structure):
    """srsgpu_pdsch_dmrs_config (include/srsgpu_phy.h): dmrs_pdsch_processor::config_t of one transmission."""
    _fields_ = [
        ("slot_index", ctypes.c_uint16),
        ("scrambling_id", ctypes.c_uint16),
        ("n_scid", ctypes.c_uint8),
        ("dmrs_type", ctypes.c_uint8),
        ("nof_layers", ctypes.c_uint8),
        ("nof_ports", ctypes.c_uint8),
        ("dmrs_symbol_mask", ctypes.c_uint16),
        ("reference_point_k_rb", ctypes.c_uint16),
        ("rb_start", ctypes.c_uint16),
        ("nof_rb", ctypes.c_uint16),
        ("amplitude", ctypes.c_float),
        ("precoding", ctypes.c_float * 32),
        ("grid_index", ctypes.c_uint32),
    ]


assert ctypes.sizeof(PdschDmrsConfig) == 152


class PuschDemodConfig(ctypes.Structure):
    """srsgpu_pusch_demod_config (include/srsgpu_phy.h): one transmission of pusch_demodulator::configuration."""
    _fields_ = [
        ("rnti", ctypes.c_uint16),
        ("n_id", ctypes.c_uint16),
        ("modulation_order", ctypes.c_uint8),
        ("nof_tx_layers", ctypes.c_uint8),
        ("nof_rx_ports", ctypes.c_uint8),
        ("start_symbol", ctypes.c_uint8),
        ("nof_symbols", ctypes.c_uint8),
        ("dmrs_type", ctypes.c_uint8),
        ("nof_cdm_groups_without_data", ctypes.c_uint8),
        ("equalizer", ctypes.c_uint8),
        ("dmrs_symbol_mask", ctypes.c_uint16),
        ("rb_start", ctypes.c_uint16),
        ("nof_rb", ctypes.c_uint16),
        ("estimate_layout", ctypes.c_uint8),
        ("cfo_compensated", ctypes.c_uint8),
        ("grid_index", ctypes.c_uint32),
        ("llr_offset", ctypes.c_uint32),
        ("numerology", ctypes.c_uint8),
        ("transform_precoding", ctypes.c_uint8),
        ("pad2", ctypes.c_uint8 * 2),
    ]


assert ctypes.sizeof(PuschDemodConfig) == 32
DEMOD_STATS = 30  # SRSGPU_DEMOD_STATS: 15 rows (symbols 0..13, then the transmission) x (SINR dB, EVM)


class UlschDemuxConfig(ctypes.Structure):
    """srsgpu_ulsch_demux_config (include/srsgpu_phy.h): ulsch_demultiplex::configuration of one transmission plus
    the CSI Part 2 size, the scrambling identity (placeholders) and the stream offsets."""
    _fields_ = [
        ("modulation_order", ctypes.c_uint8),
        ("nof_layers", ctypes.c_uint8),
        ("nof_prb", ctypes.c_uint16),
        ("start_symbol", ctypes.c_uint8),
        ("nof_symbols", ctypes.c_uint8),
        ("dmrs_symbol_mask", ctypes.c_uint16),
        ("dmrs_type", ctypes.c_uint8),
        ("nof_cdm_groups_without_data", ctypes.c_uint8),
        ("rnti", ctypes.c_uint16),
        ("n_id", ctypes.c_uint16),
        ("csi2_first_symbol", ctypes.c_uint16),
        ("nof_harq_ack_rvd", ctypes.c_uint32),
        ("nof_harq_ack_bits", ctypes.c_uint32),
        ("nof_enc_harq_ack_bits", ctypes.c_uint32),
        ("nof_csi_part1_bits", ctypes.c_uint32),
        ("nof_enc_csi_part1_bits", ctypes.c_uint32),
        ("nof_csi_part2_bits", ctypes.c_uint32),
        ("nof_enc_csi_part2_bits", ctypes.c_uint32),
        ("llr_offset", ctypes.c_uint32),
        ("sch_offset", ctypes.c_uint32),
        ("harq_offset", ctypes.c_uint32),
        ("csi1_offset", ctypes.c_uint32),
        ("csi2_offset", ctypes.c_uint32),
    ]


assert ctypes.sizeof(UlschDemuxConfig) == 64


class PuschChestConfig(ctypes.Structure):
    """srsgpu_pusch_chest_config (include/srsgpu_phy.h): dmrs_pusch_estimator::configuration of one transmission."""
    _fields_ = [
        ("scrambling_id", ctypes.c_uint16),
        ("n_scid", ctypes.c_uint8),
        ("dmrs_type", ctypes.c_uint8),
        ("nof_tx_layers", ctypes.c_uint8),
        ("nof_rx_ports", ctypes.c_uint8),
        ("start_symbol", ctypes.c_uint8),
        ("nof_symbols", ctypes.c_uint8),
        ("dmrs_symbol_mask", ctypes.c_uint16),
        ("rb_start", ctypes.c_uint16),
        ("nof_rb", ctypes.c_uint16),
        ("slot_index", ctypes.c_uint16),
        ("fd_smoothing", ctypes.c_uint8),
        ("estimate_layout", ctypes.c_uint8),
        ("td_strategy", ctypes.c_uint8),
        ("compensate_cfo", ctypes.c_uint8),
        ("scaling", ctypes.c_float),
        ("grid_index", ctypes.c_uint32),
        ("numerology", ctypes.c_uint8),
        ("dmrs_sequence", ctypes.c_uint8),
        ("pad", ctypes.c_uint8 * 2),
    ]


assert ctypes.sizeof(PuschChestConfig) == 32
CHEST_FD_NONE, CHEST_FD_MEAN, CHEST_FD_FILTER = 0, 1, 2
CHEST_TD_AVERAGE, CHEST_TD_INTERPOLATE = 0, 1
CHEST_METRICS = 8  # per (tx, port): RSRP, EPRE, noise variance, SNR, TA (s), CFO (Hz, NaN without), 0, 0
CE_PER_SYMBOL, CE_COMPACT = 0, 1  # channel-estimate layouts (SRSGPU_CE_*)
EQ_ZF, EQ_MMSE = 0, 1


class OfdmConfig(ctypes.Structure):
    """srsgpu_ofdm_config (include/srsgpu_phy.h): ofdm_modulator_configuration / ofdm_demodulator_configuration."""
    _fields_ = [
        ("numerology", ctypes.c_uint32),
        ("bw_rb", ctypes.c_uint32),
        ("dft_size", ctypes.c_uint32),
        ("cp_extended", ctypes.c_uint32),
        ("nof_samples_window_offset", ctypes.c_uint32),
        ("scale", ctypes.c_float),
        ("center_freq_hz", ctypes.c_double),
    ]


assert ctypes.sizeof(OfdmConfig) == 32

_lib = None


def load_library(path: str = LIB_PATH):
    """Loads libsrsgpu_phy.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise SrsGpuError(f"{path} not built: run srsran-5g_amd/build.sh (or __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    P = ctypes.c_void_p
    lib.srsgpu_version.restype = ctypes.c_int
    lib.srsgpu_last_error.restype = ctypes.c_char_p
    lib.srsgpu_context_create.argtypes = [ctypes.c_int, ctypes.POINTER(P)]
    lib.srsgpu_context_destroy.argtypes = [P]
    lib.srsgpu_context_destroy.restype = None
    lib.srsgpu_context_device.argtypes = [P]
    lib.srsgpu_context_device.restype = ctypes.c_int
    lib.srsgpu_context_set_option.argtypes = [P, ctypes.c_int, ctypes.c_int]
    lib.srsgpu_context_set_option.restype = ctypes.c_int
    lib.srsgpu_context_get_option.argtypes = [P, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    lib.srsgpu_context_get_option.restype = ctypes.c_int
    lib.srsgpu_ldpc_decoder_plan_create.argtypes = [P, ctypes.c_int, P, ctypes.c_uint32, ctypes.POINTER(P)]
    lib.srsgpu_ldpc_decoder_plan_execute.argtypes = [P, P, P, P, P]
    lib.srsgpu_ldpc_decoder_plan_destroy.argtypes = [P]
    lib.srsgpu_ldpc_decoder_plan_destroy.restype = None
    lib.srsgpu_ldpc_decode.argtypes = [P, ctypes.c_int, P, ctypes.c_uint32, P, P, P, P]
    lib.srsgpu_pusch_cb_plan_create.argtypes = [P, ctypes.c_int, P, ctypes.c_uint32, ctypes.POINTER(P)]
    lib.srsgpu_pusch_cb_plan_execute.argtypes = [P, P, P, P, P, P, P]
    lib.srsgpu_pusch_cb_plan_destroy.argtypes = [P]
    lib.srsgpu_pusch_cb_plan_destroy.restype = None
    lib.srsgpu_pdsch_encoder_plan_create.argtypes = [P, P, ctypes.c_uint32, ctypes.POINTER(P)]
    lib.srsgpu_pusch_decoder_plan_decoder_input_llrs.argtypes = [P]
    lib.srsgpu_pusch_decoder_plan_decoder_input_llrs.restype = ctypes.c_uint64
    lib.srsgpu_pdsch_encoder_plan_nof_codeblocks.argtypes = [P]
    lib.srsgpu_pdsch_encoder_plan_nof_codeblocks.restype = ctypes.c_uint32
    lib.srsgpu_pdsch_encoder_plan_execute.argtypes = [P, P, P, P]
    lib.srsgpu_pdsch_encoder_plan_destroy.argtypes = [P]
    lib.srsgpu_pdsch_encoder_plan_destroy.restype = None
    lib.srsgpu_pusch_decoder_plan_create.argtypes = [P, ctypes.c_int, P, ctypes.c_uint32, ctypes.POINTER(P)]
    lib.srsgpu_pusch_decoder_plan_nof_codeblocks.argtypes = [P]
    lib.srsgpu_pusch_decoder_plan_nof_codeblocks.restype = ctypes.c_uint32
    lib.srsgpu_pusch_decoder_plan_execute.argtypes = [P, P, P, P, P, P, P, P, P]
    lib.srsgpu_pusch_decoder_plan_execute_arena.argtypes = [P, P, P, P, P, P, P, P, P]
    lib.srsgpu_pusch_decoder_plan_assemble.argtypes = [P, P, P, P, P, P]
    lib.srsgpu_pusch_decoder_plan_destroy.argtypes = [P]
    lib.srsgpu_pusch_decoder_plan_destroy.restype = None
    lib.srsgpu_pdsch_modulator_plan_create.argtypes = [P, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                       ctypes.POINTER(P)]
    lib.srsgpu_pdsch_modulator_plan_create_ex.argtypes = [P, P, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                          ctypes.POINTER(P)]
    lib.srsgpu_pdsch_modulator_plan_execute.argtypes = [P, P, P, P]
    lib.srsgpu_pdsch_modulator_plan_destroy.argtypes = [P]
    lib.srsgpu_pdsch_modulator_plan_destroy.restype = None
    lib.srsgpu_pdsch_dmrs_plan_create.argtypes = [P, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                  ctypes.POINTER(P)]
    lib.srsgpu_pdsch_dmrs_plan_create_ex.argtypes = [P, P, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                     ctypes.POINTER(P)]
    lib.srsgpu_pdsch_dmrs_plan_execute.argtypes = [P, P, P]
    lib.srsgpu_pusch_demodulator_plan_create_ex.argtypes = [P, P, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                            ctypes.POINTER(P)]
    lib.srsgpu_pusch_demodulator_plan_execute_ex.argtypes = [P, P, P, P, P, P, P]
    lib.srsgpu_ulsch_demux_plan_create.argtypes = [P, P, ctypes.c_uint32, ctypes.POINTER(P)]
    lib.srsgpu_ulsch_demux_plan_nof_llrs.argtypes = [P, ctypes.c_uint32, ctypes.c_uint32]
    lib.srsgpu_ulsch_demux_plan_nof_llrs.restype = ctypes.c_uint32
    lib.srsgpu_ulsch_demux_plan_symbol_llrs.argtypes = [P, ctypes.c_uint32, ctypes.c_uint32, P]
    lib.srsgpu_ulsch_demux_plan_symbol_llrs.restype = ctypes.c_int
    lib.srsgpu_ulsch_demux_plan_execute.argtypes = [P, P, P, P, P, P, P]
    lib.srsgpu_ulsch_demux_plan_destroy.argtypes = [P]
    lib.srsgpu_ulsch_demux_plan_destroy.restype = None
    lib.srsgpu_pusch_chest_plan_create_ex.argtypes = [P, P, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                      ctypes.POINTER(P)]
    lib.srsgpu_pdsch_dmrs_plan_destroy.argtypes = [P]
    lib.srsgpu_pdsch_dmrs_plan_destroy.restype = None
    lib.srsgpu_pusch_chest_plan_create.argtypes = [P, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                   ctypes.POINTER(P)]
    lib.srsgpu_pusch_chest_plan_execute.argtypes = [P, P, P, P, P, P]
    lib.srsgpu_pusch_chest_plan_execute_copy.argtypes = [P, P, P, P, P, P, ctypes.c_uint32, ctypes.c_uint64, P]
    lib.srsgpu_pusch_chest_plan_destroy.argtypes = [P]
    lib.srsgpu_pusch_chest_plan_destroy.restype = None
    lib.srsgpu_pusch_demodulator_plan_create.argtypes = [P, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                         ctypes.POINTER(P)]
    lib.srsgpu_pusch_demodulator_plan_nof_llrs.argtypes = [P, ctypes.c_uint32]
    lib.srsgpu_pusch_demodulator_plan_nof_llrs.restype = ctypes.c_uint32
    lib.srsgpu_pusch_demodulator_plan_execute.argtypes = [P, P, P, P, P, P]
    lib.srsgpu_pusch_demodulator_plan_destroy.argtypes = [P]
    lib.srsgpu_pusch_demodulator_plan_destroy.restype = None
    for name in ("srsgpu_ofdm_modulator_plan_create", "srsgpu_ofdm_demodulator_plan_create"):
        getattr(lib, name).argtypes = [P, P, ctypes.c_uint32, ctypes.c_uint32, P, ctypes.POINTER(P)]
    for name in ("srsgpu_ofdm_modulator_symbols_plan_create", "srsgpu_ofdm_demodulator_symbols_plan_create"):
        getattr(lib, name).argtypes = [P, P] + [ctypes.c_uint32] * 4 + [ctypes.POINTER(P)]
    lib.srsgpu_ofdm_plan_nof_samples.argtypes = [P]
    lib.srsgpu_ofdm_plan_nof_samples.restype = ctypes.c_uint64
    lib.srsgpu_ofdm_plan_nof_grid_words.argtypes = [P]
    lib.srsgpu_ofdm_plan_nof_grid_words.restype = ctypes.c_uint64
    lib.srsgpu_ofdm_plan_concat.argtypes = [P, P, ctypes.c_uint32, ctypes.POINTER(P)]
    lib.srsgpu_ofdm_plan_get_jobs.argtypes = [P, P, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    lib.srsgpu_ofdm_jobs_execute.argtypes = [P, P, ctypes.c_uint32, P, P, P]
    lib.srsgpu_ofdm_jobs_execute_direct.argtypes = [P, P, ctypes.c_uint32, P]
    lib.srsgpu_copy_spans.argtypes = [P, ctypes.c_uint32, ctypes.c_uint64, P]
    if hasattr(lib, "srsgpu_merge_spans"):  # (libraries built before round 6 lack it: A/B runs of older builds)
        lib.srsgpu_merge_spans.argtypes = [P, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32, P]
    lib.srsgpu_ofdm_plan_sample_offset.argtypes = [P, ctypes.c_uint32, ctypes.c_uint32]
    lib.srsgpu_ofdm_plan_sample_offset.restype = ctypes.c_uint64
    lib.srsgpu_ofdm_modulator_plan_execute.argtypes = [P, P, P, P]
    lib.srsgpu_ofdm_demodulator_plan_execute.argtypes = [P, P, P, P]
    if hasattr(lib, "srsgpu_ofdm_modulator_plan_execute_twin"):
        lib.srsgpu_ofdm_modulator_plan_execute_twin.argtypes = [P, P, P, P, P]
    lib.srsgpu_ofdm_plan_destroy.argtypes = [P]
    lib.srsgpu_ofdm_plan_destroy.restype = None
    for name in ("srsgpu_pusch_decoder_plan", "srsgpu_pdsch_encoder_plan"):
        getattr(lib, name + "_enable_timing").argtypes = [P, ctypes.c_int]
        getattr(lib, name + "_stage_times").argtypes = [P, P, ctypes.POINTER(ctypes.c_uint32)]
    _lib = lib
    return lib


# Every symbol include/srsgpu_phy.h declares (checked by tests/test_capi_symbols.py).
EXPORTED_SYMBOLS = [
    "srsgpu_version", "srsgpu_last_error", "srsgpu_context_create", "srsgpu_context_destroy", "srsgpu_context_device",
    "srsgpu_context_set_option", "srsgpu_context_get_option", "srsgpu_pusch_demodulator_plan_scrambling",
    "srsgpu_ldpc_decoder_plan_create", "srsgpu_ldpc_decoder_plan_execute", "srsgpu_ldpc_decoder_plan_destroy",
    "srsgpu_ldpc_decode", "srsgpu_pusch_cb_plan_create", "srsgpu_pusch_cb_plan_execute",
    "srsgpu_pusch_cb_plan_destroy", "srsgpu_pdsch_encoder_plan_create", "srsgpu_pdsch_encoder_plan_nof_codeblocks",
    "srsgpu_pdsch_encoder_plan_execute", "srsgpu_pdsch_encoder_plan_destroy", "srsgpu_pusch_decoder_plan_create",
    "srsgpu_pusch_decoder_plan_nof_codeblocks", "srsgpu_pusch_decoder_plan_decoder_input_llrs",
    "srsgpu_pusch_decoder_plan_execute", "srsgpu_pusch_decoder_plan_execute_arena",
    "srsgpu_pusch_decoder_plan_assemble",
    "srsgpu_pusch_decoder_plan_destroy", "srsgpu_pusch_decoder_plan_enable_timing",
    "srsgpu_pusch_decoder_plan_stage_times", "srsgpu_pdsch_encoder_plan_enable_timing",
    "srsgpu_pdsch_encoder_plan_stage_times", "srsgpu_pdsch_modulator_plan_create",
    "srsgpu_pdsch_modulator_plan_create_ex", "srsgpu_pdsch_modulator_plan_execute", "srsgpu_pdsch_modulator_plan_destroy",
    "srsgpu_ofdm_modulator_plan_create", "srsgpu_ofdm_demodulator_plan_create", "srsgpu_ofdm_plan_nof_samples",
    "srsgpu_ofdm_modulator_symbols_plan_create", "srsgpu_ofdm_demodulator_symbols_plan_create", "srsgpu_harq_copy",
    "srsgpu_ofdm_plan_sample_offset", "srsgpu_ofdm_modulator_plan_execute", "srsgpu_ofdm_demodulator_plan_execute",
    "srsgpu_ofdm_modulator_plan_execute_twin",
    "srsgpu_ofdm_plan_concat", "srsgpu_ofdm_plan_nof_grid_words", "srsgpu_ofdm_plan_get_jobs",
    "srsgpu_ofdm_jobs_execute", "srsgpu_ofdm_jobs_execute_direct", "srsgpu_copy_spans", "srsgpu_merge_spans",
    "srsgpu_ofdm_plan_destroy", "srsgpu_pusch_demodulator_plan_create", "srsgpu_pusch_demodulator_plan_nof_llrs",
    "srsgpu_pusch_demodulator_plan_execute", "srsgpu_pusch_demodulator_plan_destroy",
    "srsgpu_pusch_demodulator_plan_create_ex", "srsgpu_pusch_demodulator_plan_execute_ex",
    "srsgpu_pusch_chest_plan_create_ex", "srsgpu_ulsch_demux_plan_create", "srsgpu_ulsch_demux_plan_nof_llrs",
    "srsgpu_ulsch_demux_plan_symbol_llrs", "srsgpu_harq_copy_arenas",
    "srsgpu_ulsch_demux_plan_execute", "srsgpu_ulsch_demux_plan_destroy",
    "srsgpu_pusch_chest_plan_create", "srsgpu_pusch_chest_plan_execute", "srsgpu_pusch_chest_plan_destroy",
    "srsgpu_pusch_chest_plan_execute_copy",
    "srsgpu_pdsch_dmrs_plan_create", "srsgpu_pdsch_dmrs_plan_create_ex", "srsgpu_pdsch_dmrs_plan_execute", "srsgpu_pdsch_dmrs_plan_destroy",
]


def _stage_times(prefix, handle, n):
    ms = (ctypes.c_float * n)()
    cnt = ctypes.c_uint32()
    _check(getattr(_lib, prefix + "_stage_times")(handle, ctypes.cast(ms, ctypes.c_void_p), ctypes.byref(cnt)))
    return list(ms), cnt.value


def _check(rc: int):
    if rc != SRSGPU_OK:
        raise SrsGpuError(f"srsgpu error {rc}: {_lib.srsgpu_last_error().decode()}")


def _stream_handle(stream) -> Optional[int]:
    if stream is None:
        return torch.cuda.current_stream().cuda_stream if torch is not None else None
    if hasattr(stream, "cuda_stream"):
        return stream.cuda_stream
    return int(stream)


def span_list(spans):
    """The srsgpu_copy_span array of spans = [(src tensor, dst tensor)] (contiguous device tensors of the same byte
    size, a multiple of 16) on the device, and its byte counts."""
    arr = np.zeros(len(spans), np.dtype([("src", "<u8"), ("dst", "<u8"), ("bytes", "<u8")]))
    for i, (a, b) in enumerate(spans):
        n = a.numel() * a.element_size()
        if n != b.numel() * b.element_size():
            raise SrsGpuError("copy_spans: source and destination sizes differ")
        arr[i] = (_dptr(a), _dptr(b), n)
    return torch.from_numpy(arr.view(np.uint8).copy()).to(spans[0][0].device), arr["bytes"]


def copy_spans(spans, stream=None):
    """srsgpu_copy_spans: spans = [(src tensor, dst tensor)], each a contiguous device tensor of the same byte size (a
    multiple of 16). One launch copies them all."""
    d, nbytes = span_list(spans)
    _check(_lib.srsgpu_copy_spans(_dptr(d), len(spans), int(nbytes.max()), _stream_handle(stream)))
    return d  # keep alive until the stream has run the copies


def merge_spans(spans, sentinel=0xFFFFFFFF, stream=None):
    """srsgpu_merge_spans: as copy_spans, but a 32-bit source word replaces the destination's only when it is not
    `sentinel` (the multi-device PDSCH batch's gather of sentinel-filled shard grids)."""
    d, nbytes = span_list(spans)
    _check(_lib.srsgpu_merge_spans(_dptr(d), len(spans), int(nbytes.max()), int(sentinel), _stream_handle(stream)))
    return d


def _dptr(t) -> int:
    if t is None:
        return None
    if not t.is_cuda:
        raise SrsGpuError("expected a device (HIP) tensor")
    if not t.is_contiguous():
        raise SrsGpuError("expected a contiguous tensor")
    return t.data_ptr()


# srsgpu_option (include/srsgpu_phy.h): kernel-selection options of a context, read at plan creation.
OPTION_DECODER_SPLIT = 1          # -1 auto (default), 0 one-row-pair kernel, 1 edge-split kernel
OPTION_DECODER_PAIRS = 2          # 0 (default) / 1: Z = 144..192 codeblocks two per workgroup
OPTION_DECODER_FUSED_DEMATCH = 3  # 1 (default) / 0: every codeblock through the separate rate dematcher
OPTION_ENCODER_BYTE_KERNEL = 4    # 0 (default) / 1: the byte-per-bit encoder kernel for every codeblock
OPTION_ENCODER_ZERO_OUTPUT = 5    # 0 (default) / 1: the encoder always clears its output first
OPTION_DEFAULTS = {OPTION_DECODER_SPLIT: -1, OPTION_DECODER_PAIRS: 0, OPTION_DECODER_FUSED_DEMATCH: 1,
                   OPTION_ENCODER_BYTE_KERNEL: 0, OPTION_ENCODER_ZERO_OUTPUT: 0}


class Context:
    """srsgpu_context: one per GPU (one process per GPU)."""

    def __init__(self, device: int = 0):
        lib = load_library()
        if torch is None or not torch.cuda.is_available():
            raise SrsGpuError("no HIP device available (the srsgpu kernels need an MI355X)")
        self.device = device
        h = ctypes.c_void_p()
        _check(lib.srsgpu_context_create(device, ctypes.byref(h)))
        self.handle = h

    def set_option(self, option: int, value: int) -> None:
        """srsgpu_context_set_option: plans created afterwards use it."""
        _check(_lib.srsgpu_context_set_option(self.handle, option, value))

    def get_option(self, option: int) -> int:
        v = ctypes.c_int()
        _check(_lib.srsgpu_context_get_option(self.handle, option, ctypes.byref(v)))
        return v.value

    def options(self, **kw):
        """Context manager: the given options (OPTION_* names without the prefix, lower case) while inside, the
        previous values after."""
        import contextlib

        @contextlib.contextmanager
        def scope():
            keys = {globals()["OPTION_" + k.upper()]: v for k, v in kw.items()}
            old = {k: self.get_option(k) for k in keys}
            try:
                for k, v in keys.items():
                    self.set_option(k, v)
                yield self
            finally:
                for k, v in old.items():
                    self.set_option(k, v)
        return scope()

    def close(self):
        if getattr(self, "handle", None):
            _lib.srsgpu_context_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


@dataclass
class CodeblockDecodeConfig:
    """Mirror of srsran::ldpc_decoder::configuration (ldpc_decoder.h:44) for one codeblock."""
    base_graph: int
    lifting_size: int
    nof_crc_bits: int = 16
    nof_filler_bits: int = 0
    max_iterations: int = 6
    scaling_factor: float = 0.8


def make_configs(cfgs: Sequence[CodeblockDecodeConfig], nof_llrs: Sequence[int], crc_polys: Sequence[int],
                 llr_offsets: Optional[Sequence[int]] = None, out_offsets: Optional[Sequence[int]] = None):
    """Packs per-codeblock configurations into the C array, with default contiguous offsets."""
    n = len(cfgs)
    arr = (LdpcDecoderConfig * n)()
    llr_off = 0
    out_off = 0
    for i, c in enumerate(cfgs):
        a = arr[i]
        a.base_graph = c.base_graph
        a.crc_poly = crc_polys[i]
        a.lifting_size = c.lifting_size
        a.nof_filler_bits = c.nof_filler_bits
        a.nof_crc_bits = c.nof_crc_bits
        a.max_iterations = c.max_iterations
        a.scaling_factor = c.scaling_factor
        a.nof_llrs = nof_llrs[i]
        a.llr_offset = llr_offsets[i] if llr_offsets is not None else llr_off
        a.out_offset = out_offsets[i] if out_offsets is not None else out_off
        llr_off += nof_llrs[i]
        out_off += (BG_K[c.base_graph] * c.lifting_size + 7) // 8
    return arr


class LdpcDecoderPlan:
    """srsgpu_ldpc_decoder_plan: validated, device-resident batch of decoder work (hipGraph-capturable execute)."""

    def __init__(self, ctx: Context, impl: int, cfg_array):
        self.ctx = ctx
        h = ctypes.c_void_p()
        _check(_lib.srsgpu_ldpc_decoder_plan_create(ctx.handle, impl, ctypes.cast(cfg_array, ctypes.c_void_p),
                                                    len(cfg_array), ctypes.byref(h)))
        self.handle = h
        self.nof_cbs = len(cfg_array)

    def execute(self, d_llrs, d_out, d_iters, stream=None):
        _check(_lib.srsgpu_ldpc_decoder_plan_execute(self.handle, _dptr(d_llrs), _dptr(d_out), _dptr(d_iters),
                                                     _stream_handle(stream)))

    def close(self):
        if getattr(self, "handle", None):
            _lib.srsgpu_ldpc_decoder_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def unpack_bits(packed: np.ndarray, nbits: int) -> np.ndarray:
    return np.unpackbits(np.asarray(packed, dtype=np.uint8))[:nbits]


class LdpcDecoder:
    """GPU implementation of srsran::ldpc_decoder (ldpc_decoder.h), created like
    create_ldpc_decoder_factory_sw(type)->create() (channel_coding_factories.h): type "generic" or "avx2"/"avx512"/
    "neon"/"auto" selects the arithmetic variant the results are bit-exact with."""

    def __init__(self, ctx: Context, dec_type: str = "auto"):
        if dec_type not in IMPL_BY_NAME:
            raise SrsGpuError(f"invalid LDPC decoder type '{dec_type}'")
        self.ctx = ctx
        self.impl = IMPL_BY_NAME[dec_type]

    def decode(self, llrs: np.ndarray, cfg: CodeblockDecodeConfig, crc_poly: Optional[int] = None,
               output_init: Optional[np.ndarray] = None):
        """Decodes one codeblock. Returns (nof_iterations or None, K*Z unpacked bits) like ldpc_decoder::decode."""
        res = self.decode_batch([llrs], [cfg], [crc_poly], None if output_init is None else [output_init])
        return res[0]

    def decode_batch(self, llrs_list: List[np.ndarray], cfgs: List[CodeblockDecodeConfig],
                     crc_polys: List[Optional[int]], output_inits=None):
        n = len(cfgs)
        nof_llrs = [int(np.asarray(x).size) for x in llrs_list]
        polys = [CRC_NONE if p is None else p for p in crc_polys]
        arr = make_configs(cfgs, nof_llrs, polys)
        flat = np.concatenate([np.asarray(x, dtype=np.int8) for x in llrs_list]) if n else np.zeros(0, np.int8)
        out_bytes = [(BG_K[c.base_graph] * c.lifting_size + 7) // 8 for c in cfgs]
        dev = torch.device("cuda", self.ctx.device)
        d_llrs = torch.from_numpy(flat).to(dev)
        if output_inits is not None:
            init = np.concatenate([np.packbits(np.asarray(o, dtype=np.uint8)) for o in output_inits])
            d_out = torch.from_numpy(init).to(dev)
        else:
            d_out = torch.zeros(sum(out_bytes), dtype=torch.uint8, device=dev)
        d_iters = torch.zeros(n, dtype=torch.int32, device=dev)
        stream = torch.cuda.current_stream(dev)
        _check(_lib.srsgpu_ldpc_decode(self.ctx.handle, self.impl, ctypes.cast(arr, ctypes.c_void_p), n,
                                       _dptr(d_llrs), _dptr(d_out), _dptr(d_iters), stream.cuda_stream))
        out = d_out.cpu().numpy()
        iters = d_iters.cpu().numpy()
        results = []
        off = 0
        for i, c in enumerate(cfgs):
            nb = BG_K[c.base_graph] * c.lifting_size
            bits = unpack_bits(out[off: off + out_bytes[i]], nb)
            off += out_bytes[i]
            results.append((None if iters[i] < 0 else int(iters[i]), bits))
        return results


class PuschCbPlan:
    """srsgpu_pusch_cb_plan: rate dematching + HARQ combining + LDPC decoding + CB CRC for a batch of codeblocks."""

    def __init__(self, ctx: Context, impl: int, cfg_array):
        self.ctx = ctx
        h = ctypes.c_void_p()
        _check(_lib.srsgpu_pusch_cb_plan_create(ctx.handle, impl, ctypes.cast(cfg_array, ctypes.c_void_p),
                                                len(cfg_array), ctypes.byref(h)))
        self.handle = h
        self.nof_cbs = len(cfg_array)

    def execute(self, d_llrs, d_harq, d_out, d_iters, d_cb_crc_ok=None, stream=None):
        _check(_lib.srsgpu_pusch_cb_plan_execute(self.handle, _dptr(d_llrs), _dptr(d_harq), _dptr(d_out),
                                                 _dptr(d_iters), _dptr(d_cb_crc_ok), _stream_handle(stream)))

    def close(self):
        if getattr(self, "handle", None):
            _lib.srsgpu_pusch_cb_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


@dataclass
class PuschCodeblock:
    """One codeblock of a PUSCH transport block: hw_pusch_decoder_configuration (hw_accelerator_pusch_dec.h:30)."""
    base_graph: int
    lifting_size: int
    rv: int
    modulation_order: int
    rm_length: int
    nof_filler_bits: int = 0
    crc_poly: int = CRC24B
    nof_crc_bits: int = 24
    Nref: int = 0
    new_data: bool = True
    use_early_stop: bool = True
    max_iterations: int = 6
    scaling_factor: float = 0.8


def make_pusch_cb_configs(cbs: Sequence[PuschCodeblock]):
    """Packs codeblocks with contiguous LLR / HARQ / output offsets."""
    arr = (PuschCbConfig * len(cbs))()
    lo = ho = oo = 0
    for i, c in enumerate(cbs):
        a = arr[i]
        a.base_graph, a.rv, a.modulation_order, a.crc_poly = c.base_graph, c.rv, c.modulation_order, c.crc_poly
        a.lifting_size, a.nof_filler_bits, a.nof_crc_bits = c.lifting_size, c.nof_filler_bits, c.nof_crc_bits
        a.max_iterations, a.new_data, a.use_early_stop = c.max_iterations, int(c.new_data), int(c.use_early_stop)
        a.scaling_factor, a.Nref, a.rm_length = c.scaling_factor, c.Nref, c.rm_length
        a.llr_offset, a.harq_offset, a.out_offset = lo, ho, oo
        lo += c.rm_length
        ho += BG_N_SHORT[c.base_graph] * c.lifting_size
        oo += (BG_K[c.base_graph] * c.lifting_size + 7) // 8
    return arr, lo, ho, oo


class PuschCodeblockDecoder:
    """GPU counterpart of pusch_codeblock_decoder (pusch_codeblock_decoder.cpp:33) / hw_accelerator_pusch_dec with an
    external (device-resident) HARQ buffer: the caller owns d_harq and d_cb_crc_ok across retransmissions."""

    def __init__(self, ctx: Context, dec_type: str = "auto"):
        if dec_type not in IMPL_BY_NAME:
            raise SrsGpuError(f"invalid decoder type '{dec_type}'")
        self.ctx = ctx
        self.impl = IMPL_BY_NAME[dec_type]

    def decode(self, llrs_list, cbs: Sequence[PuschCodeblock], harq: np.ndarray = None, cb_crc_ok: np.ndarray = None):
        """Returns (results [(nof_iterations or None, K*Z bits)], updated harq buffer, updated crc flags)."""
        arr, nllr, nharq, nout = make_pusch_cb_configs(cbs)
        dev = torch.device("cuda", self.ctx.device)
        flat = np.concatenate([np.asarray(x, dtype=np.int8) for x in llrs_list])
        assert flat.size == nllr
        d_llrs = torch.from_numpy(flat).to(dev)
        d_harq = (torch.from_numpy(np.asarray(harq, dtype=np.int8).copy()).to(dev) if harq is not None
                  else torch.zeros(nharq, dtype=torch.int8, device=dev))
        d_crc = (torch.from_numpy(np.asarray(cb_crc_ok, dtype=np.uint8).copy()).to(dev) if cb_crc_ok is not None
                 else torch.zeros(len(cbs), dtype=torch.uint8, device=dev))
        d_out = torch.zeros(nout, dtype=torch.uint8, device=dev)
        d_iters = torch.zeros(len(cbs), dtype=torch.int32, device=dev)
        plan = PuschCbPlan(self.ctx, self.impl, arr)
        plan.execute(d_llrs, d_harq, d_out, d_iters, d_crc)
        torch.cuda.synchronize(dev)
        plan.close()
        out = d_out.cpu().numpy()
        iters = d_iters.cpu().numpy()
        res = []
        off = 0
        for i, c in enumerate(cbs):
            nb = BG_K[c.base_graph] * c.lifting_size
            ob = (nb + 7) // 8
            res.append((None if iters[i] < 0 else int(iters[i]), unpack_bits(out[off:off + ob], nb)))
            off += ob
        return res, d_harq.cpu().numpy(), d_crc.cpu().numpy()


@dataclass
class PdschTransportBlock:
    """pdsch_encoder::configuration (pdsch_encoder.h) of one transport block."""
    base_graph: int
    rv: int
    modulation_order: int
    nof_layers: int
    nof_ch_symbols: int
    Nref: int = 0


def make_pdsch_configs(tbs_bytes: Sequence[int], tbs: Sequence[PdschTransportBlock]):
    """Packs transport blocks with contiguous TB / codeword (word-aligned) offsets."""
    arr = (PdschTbConfig * len(tbs))()
    to = co = 0
    cw_offsets = []
    for i, (nb, t) in enumerate(zip(tbs_bytes, tbs)):
        a = arr[i]
        a.base_graph, a.rv, a.modulation_order, a.nof_layers = t.base_graph, t.rv, t.modulation_order, t.nof_layers
        a.tbs_bytes, a.nof_ch_symbols, a.Nref, a.tb_offset, a.cw_offset = nb, t.nof_ch_symbols, t.Nref, to, co
        cw_offsets.append(co)
        to += nb
        co += (t.nof_ch_symbols * t.modulation_order + 31) // 32 * 4
    return arr, to, co, cw_offsets


class PdschEncoderPlan:
    """srsgpu_pdsch_encoder_plan: TB CRC + segmentation + CB CRC + LDPC + rate matching of a slot's TBs."""

    def __init__(self, ctx: Context, cfg_array):
        self.ctx = ctx
        h = ctypes.c_void_p()
        _check(_lib.srsgpu_pdsch_encoder_plan_create(ctx.handle, ctypes.cast(cfg_array, ctypes.c_void_p),
                                                     len(cfg_array), ctypes.byref(h)))
        self.handle = h
        self.nof_tbs = len(cfg_array)
        self.nof_codeblocks = int(_lib.srsgpu_pdsch_encoder_plan_nof_codeblocks(h))

    def execute(self, d_tbs, d_codewords, stream=None):
        _check(_lib.srsgpu_pdsch_encoder_plan_execute(self.handle, _dptr(d_tbs), _dptr(d_codewords),
                                                      _stream_handle(stream)))

    def enable_timing(self, enable=True):
        _check(_lib.srsgpu_pdsch_encoder_plan_enable_timing(self.handle, int(enable)))

    def stage_times(self):
        """([ms TB CRC, ms encode], number of executes) accumulated since the previous call."""
        return _stage_times("srsgpu_pdsch_encoder_plan", self.handle, 2)

    def close(self):
        if getattr(self, "handle", None):
            _lib.srsgpu_pdsch_encoder_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class PdschEncoder:
    """GPU counterpart of srsran::pdsch_encoder (pdsch_encoder_impl.cpp:28); encode() returns the codeword unpacked
    one bit per byte like the reference."""

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def encode_batch(self, tbs: Sequence[np.ndarray], cfgs: Sequence[PdschTransportBlock]):
        arr, ntb, ncw, cw_offsets = make_pdsch_configs([t.size for t in tbs], cfgs)
        dev = torch.device("cuda", self.ctx.device)
        d_tbs = torch.from_numpy(np.concatenate([np.asarray(t, np.uint8) for t in tbs])).to(dev)
        d_cw = torch.full((max(ncw, 4),), 0xAB, dtype=torch.uint8, device=dev)
        plan = PdschEncoderPlan(self.ctx, arr)
        plan.execute(d_tbs, d_cw)
        torch.cuda.synchronize(dev)
        plan.close()
        cw = d_cw.cpu().numpy()
        out = []
        for off, c in zip(cw_offsets, cfgs):
            G = c.nof_ch_symbols * c.modulation_order
            out.append(np.unpackbits(cw[off: off + (G + 7) // 8])[:G])
        return out

    def encode(self, tb: np.ndarray, cfg: PdschTransportBlock) -> np.ndarray:
        return self.encode_batch([tb], [cfg])[0]


@dataclass
class PdschModulation:
    """pdsch_modulator::config_t (pdsch_modulator.h:38) of one transmission: contiguous non-interleaved VRB allocation
    [rb_start, rb_start + nof_rb) of the BWP and wideband precoding `weights` (nof_ports x nof_layers complex), or the
    general form: `crb_mask` (one byte per grid CRB, alloc.vrb_to_crb_mask of any type-0 / type-1 / interleaved
    allocation), `reserved` RE patterns (alloc.ReservedPattern: SSB, CSI-RS, ...) and per-PRG precoding
    (`prg_size` PRBs per PRG, `prg_weights` nof_prg x nof_ports x nof_layers complex)."""
    rnti: int
    n_id: int
    modulation_order: int
    nof_layers: int
    nof_ports: int
    bwp_start_rb: int
    bwp_size_rb: int
    rb_start: int
    nof_rb: int
    start_symbol: int
    nof_symbols: int
    dmrs_symbol_mask: int
    dmrs_type: int
    nof_cdm_groups_without_data: int
    scaling: float
    weights: np.ndarray
    crb_mask: Optional[np.ndarray] = None
    reserved: Sequence = ()
    prg_size: int = 0
    prg_weights: Optional[np.ndarray] = None

    def is_general(self) -> bool:
        return self.crb_mask is not None or len(self.reserved) > 0 or self.prg_size > 0

    def nof_re(self, grid_nof_prb: Optional[int] = None) -> int:
        if self.is_general():
            from . import alloc
            n = grid_nof_prb if grid_nof_prb is not None else self.bwp_start_rb + self.bwp_size_rb
            crbs = self.crb_mask
            if crbs is None:
                crbs = np.zeros(n, np.uint8)
                crbs[self.bwp_start_rb + self.rb_start:self.bwp_start_rb + self.rb_start + self.nof_rb] = 1
            return alloc.count_data_res(n, np.asarray(crbs)[:n], self.start_symbol, self.nof_symbols,
                                        self.dmrs_symbol_mask, self.dmrs_type, self.nof_cdm_groups_without_data,
                                        self.bwp_start_rb, self.bwp_size_rb, self.reserved)
        dm = (4 if self.dmrs_type == 2 else 6) * self.nof_cdm_groups_without_data
        return sum((12 - dm if (self.dmrs_symbol_mask >> l) & 1 else 12) * self.nof_rb
                   for l in range(self.start_symbol, self.start_symbol + self.nof_symbols))


def make_alloc_exts(mods, grid_nof_prb: int):
    """srsgpu_alloc_ext array of the general transmissions (None when every one is contiguous and wideband); the
    returned keep-alive list holds the buffers the structures point to until the plan is created."""
    if not any(m.is_general() for m in mods):
        return None, []
    exts = (AllocExtC * len(mods))()
    keep = []
    for i, m in enumerate(mods):
        if not m.is_general():
            continue
        e = exts[i]
        if m.crb_mask is not None:
            c = np.zeros(grid_nof_prb, np.uint8)
            src = np.asarray(m.crb_mask, np.uint8)[:grid_nof_prb]
            c[:src.size] = src
            keep.append(c)
            e.crb_mask = c.ctypes.data
        if len(m.reserved):
            pats = (RePatternC * len(m.reserved))()
            for j, r in enumerate(m.reserved):
                pats[j].re_mask, pats[j].symbol_mask = r.re_mask, r.symbol_mask
                if r.crb_mask is not None:
                    c = np.zeros(grid_nof_prb, np.uint8)
                    src = np.asarray(r.crb_mask, np.uint8)[:grid_nof_prb]
                    c[:src.size] = src
                    keep.append(c)
                    pats[j].crb_mask = c.ctypes.data
            keep.append(pats)
            e.reserved, e.nof_reserved = ctypes.cast(pats, ctypes.c_void_p), len(m.reserved)
        if m.prg_size > 0:
            w = np.ascontiguousarray(np.asarray(m.prg_weights, np.complex64).reshape(-1, m.nof_ports, m.nof_layers))
            keep.append(w)
            e.prg_size, e.nof_prg, e.prg_weights = m.prg_size, w.shape[0], w.ctypes.data
    return exts, keep


def make_pdsch_mod_configs(mods: Sequence[PdschModulation], cw_offsets: Sequence[int], grid_index: Sequence[int],
                           grid_nof_prb: Optional[int] = None):
    arr = (PdschModConfig * len(mods))()
    for i, (m, off, g) in enumerate(zip(mods, cw_offsets, grid_index)):
        a = arr[i]
        a.rnti, a.n_id, a.modulation_order, a.nof_layers, a.nof_ports = (m.rnti, m.n_id, m.modulation_order,
                                                                         m.nof_layers, m.nof_ports)
        a.start_symbol, a.nof_symbols, a.dmrs_type = m.start_symbol, m.nof_symbols, m.dmrs_type
        a.nof_cdm_groups_without_data, a.dmrs_symbol_mask = m.nof_cdm_groups_without_data, m.dmrs_symbol_mask
        a.bwp_start_rb, a.bwp_size_rb, a.rb_start, a.nof_rb = m.bwp_start_rb, m.bwp_size_rb, m.rb_start, m.nof_rb
        a.scaling = m.scaling
        w = np.zeros((4, 4, 2), np.float32)
        wc = np.asarray(m.weights, np.complex64).reshape(m.nof_ports, m.nof_layers)
        w[:m.nof_ports, :m.nof_layers, 0] = wc.real
        w[:m.nof_ports, :m.nof_layers, 1] = wc.imag
        a.precoding[:] = w.reshape(-1).tolist()
        a.cw_offset, a.nof_bits, a.grid_index = off, m.nof_re(grid_nof_prb) * m.nof_layers * m.modulation_order, g
    return arr


class PdschModulatorPlan:
    """srsgpu_pdsch_modulator_plan: scrambling, modulation, layer mapping, precoding and RE mapping of a batch of
    PDSCH transmissions into bf16 resource grids (grid_nof_ports x 14 x 12 * grid_nof_prb, uint32 re | im << 16)."""

    def __init__(self, ctx: Context, cfg_array, grid_nof_prb: int, grid_nof_ports: int = 4, exts=None):
        self.ctx = ctx
        h = ctypes.c_void_p()
        if exts is None:
            _check(_lib.srsgpu_pdsch_modulator_plan_create(ctx.handle, ctypes.cast(cfg_array, ctypes.c_void_p),
                                                           len(cfg_array), grid_nof_prb, grid_nof_ports,
                                                           ctypes.byref(h)))
        else:
            _check(_lib.srsgpu_pdsch_modulator_plan_create_ex(ctx.handle, ctypes.cast(cfg_array, ctypes.c_void_p),
                                                              ctypes.cast(exts, ctypes.c_void_p), len(cfg_array),
                                                              grid_nof_prb, grid_nof_ports, ctypes.byref(h)))
        self.handle = h
        self.grid_nof_prb, self.grid_nof_ports = grid_nof_prb, grid_nof_ports

    def grid_elements(self) -> int:
        return self.grid_nof_ports * 14 * 12 * self.grid_nof_prb

    def execute(self, d_codewords, d_grids, stream=None):
        _check(_lib.srsgpu_pdsch_modulator_plan_execute(self.handle, _dptr(d_codewords), _dptr(d_grids),
                                                        _stream_handle(stream)))

    def close(self):
        if getattr(self, "handle", None):
            _lib.srsgpu_pdsch_modulator_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class PdschModulator:
    """GPU counterpart of srsran::pdsch_modulator::modulate(grid, codewords, config) (pdsch_modulator_impl.cpp:107):
    modulate() takes the packed codeword and returns the grid as uint16 bf16 bit patterns (ports, 14, nsc, 2), written
    over `grid` (or zeros) at the PDSCH REs only."""

    def __init__(self, ctx: Context, grid_nof_prb: int, grid_nof_ports: int = 4):
        self.ctx, self.grid_nof_prb, self.grid_nof_ports = ctx, grid_nof_prb, grid_nof_ports

    def modulate_batch(self, codewords: Sequence[np.ndarray], mods: Sequence[PdschModulation], grid_index=None,
                       grids: np.ndarray = None):
        dev = torch.device("cuda", self.ctx.device)
        offs, buf, o = [], [], 0
        for cw in codewords:
            b = np.asarray(cw, np.uint8)
            pad = (-b.size) % 4
            buf.append(np.concatenate([b, np.zeros(pad, np.uint8)]))
            offs.append(o)
            o += b.size + pad
        grid_index = list(range(len(mods))) if grid_index is None else list(grid_index)
        ngrids = max(grid_index) + 1 if grid_index else 1
        arr = make_pdsch_mod_configs(mods, offs, grid_index, self.grid_nof_prb)
        exts, _keep = make_alloc_exts(mods, self.grid_nof_prb)
        plan = PdschModulatorPlan(self.ctx, arr, self.grid_nof_prb, self.grid_nof_ports, exts)
        shape = (ngrids, self.grid_nof_ports, 14, 12 * self.grid_nof_prb, 2)
        g0 = np.zeros(shape, np.uint16) if grids is None else np.ascontiguousarray(grids, np.uint16).reshape(shape)
        d_grid = torch.from_numpy(g0.view(np.uint32).reshape(-1).view(np.int32)).to(dev)
        d_cw = torch.from_numpy(np.concatenate(buf) if buf else np.zeros(4, np.uint8)).to(dev)
        plan.execute(d_cw, d_grid)
        torch.cuda.synchronize(dev)
        plan.close()
        return d_grid.cpu().numpy().view(np.uint16).reshape(shape)

    def modulate(self, codeword: np.ndarray, mod: PdschModulation, grid: np.ndarray = None) -> np.ndarray:
        return self.modulate_batch([codeword], [mod], grids=None if grid is None else grid[None])[0]


@dataclass
class PdschDmrs:
    """dmrs_pdsch_processor::config_t (dmrs_pdsch_processor.h:38): contiguous CRB allocation (or `crb_mask`, one byte
    per grid CRB: rb_mask of any type-0 / interleaved allocation), DM-RS ports 0..nof_layers-1, wideband precoding
    weights (nof_ports x nof_layers complex)."""
    slot_index: int
    scrambling_id: int
    n_scid: int
    dmrs_type: int
    nof_layers: int
    nof_ports: int
    dmrs_symbol_mask: int
    reference_point_k_rb: int
    rb_start: int
    nof_rb: int
    amplitude: float
    weights: np.ndarray
    crb_mask: Optional[np.ndarray] = None

    def is_general(self) -> bool:
        return self.crb_mask is not None


def make_crb_mask_exts(dmrs, grid_nof_prb: int):
    """srsgpu_alloc_ext array carrying CRB masks only (PDSCH DM-RS, PUSCH demodulator / estimator: objects with a
    `crb_mask`; None when every allocation is contiguous) + keep-alive list."""
    if not any(d.crb_mask is not None for d in dmrs):
        return None, []
    exts = (AllocExtC * len(dmrs))()
    keep = []
    for i, d in enumerate(dmrs):
        if d.crb_mask is not None:
            c = np.zeros(grid_nof_prb, np.uint8)
            src = np.asarray(d.crb_mask, np.uint8)[:grid_nof_prb]
            c[:src.size] = src
            keep.append(c)
            exts[i].crb_mask = c.ctypes.data
    return exts, keep


make_dmrs_exts = make_crb_mask_exts


def make_pdsch_dmrs_configs(dmrs: Sequence[PdschDmrs], grid_index: Sequence[int]):
    arr = (PdschDmrsConfig * len(dmrs))()
    for i, (m, g) in enumerate(zip(dmrs, grid_index)):
        a = arr[i]
        a.slot_index, a.scrambling_id, a.n_scid, a.dmrs_type = m.slot_index, m.scrambling_id, m.n_scid, m.dmrs_type
        a.nof_layers, a.nof_ports, a.dmrs_symbol_mask = m.nof_layers, m.nof_ports, m.dmrs_symbol_mask
        a.reference_point_k_rb, a.rb_start, a.nof_rb, a.amplitude = (m.reference_point_k_rb, m.rb_start, m.nof_rb,
                                                                      m.amplitude)
        w = np.zeros((4, 4, 2), np.float32)
        wc = np.asarray(m.weights, np.complex64).reshape(m.nof_ports, m.nof_layers)
        w[:m.nof_ports, :m.nof_layers, 0] = wc.real
        w[:m.nof_ports, :m.nof_layers, 1] = wc.imag
        a.precoding[:] = w.reshape(-1).tolist()
        a.grid_index = g
    return arr


class PdschDmrsPlan:
    """srsgpu_pdsch_dmrs_plan: PDSCH DM-RS generation, cover codes, precoding and mapping into bf16 grids."""

    def __init__(self, ctx: Context, cfg_array, grid_nof_prb: int, grid_nof_ports: int = 4, exts=None):
        self.ctx = ctx
        h = ctypes.c_void_p()
        if exts is None:
            _check(_lib.srsgpu_pdsch_dmrs_plan_create(ctx.handle, ctypes.cast(cfg_array, ctypes.c_void_p),
                                                      len(cfg_array), grid_nof_prb, grid_nof_ports, ctypes.byref(h)))
        else:
            _check(_lib.srsgpu_pdsch_dmrs_plan_create_ex(ctx.handle, ctypes.cast(cfg_array, ctypes.c_void_p),
                                                         ctypes.cast(exts, ctypes.c_void_p), len(cfg_array),
                                                         grid_nof_prb, grid_nof_ports, ctypes.byref(h)))
        self.handle = h

    def execute(self, d_grids, stream=None):
        _check(_lib.srsgpu_pdsch_dmrs_plan_execute(self.handle, _dptr(d_grids), _stream_handle(stream)))

    def close(self):
        if getattr(self, "handle", None):
            _lib.srsgpu_pdsch_dmrs_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


@dataclass
class PuschDemodulation:
    """pusch_demodulator::configuration (pusch_demodulator.h:51) of one transmission, rx ports 0..nof_rx_ports-1: a
    contiguous CRB allocation [rb_start, rb_start + nof_rb) or `crb_mask` (rb_mask, one byte per grid CRB), and
    optionally transform precoding (enable_transform_precoding, one layer)."""
    rnti: int
    n_id: int
    modulation_order: int
    nof_tx_layers: int
    nof_rx_ports: int
    start_symbol: int
    nof_symbols: int
    dmrs_symbol_mask: int
    dmrs_type: int
    nof_cdm_groups_without_data: int
    rb_start: int
    nof_rb: int
    equalizer: int = EQ_ZF
    estimate_layout: int = CE_PER_SYMBOL
    cfo_compensated: int = 0  # compact layout written with CFO compensation (the estimator's compensate_cfo)
    numerology: int = 1
    crb_mask: Optional[np.ndarray] = None
    transform_precoding: int = 0

    def nof_llrs(self) -> int:
        dm = (4 if self.dmrs_type == 2 else 6) * self.nof_cdm_groups_without_data
        nrb = int(np.count_nonzero(self.crb_mask)) if self.crb_mask is not None else self.nof_rb
        nre = sum((12 - dm if (self.dmrs_symbol_mask >> l) & 1 else 12) * nrb
                  for l in range(self.start_symbol, self.start_symbol + self.nof_symbols))
        return nre * self.nof_tx_layers * self.modulation_order


def make_pusch_demod_configs(demods: Sequence[PuschDemodulation], grid_index: Sequence[int], llr_offsets=None):
    arr = (PuschDemodConfig * len(demods))()
    off = 0
    offs = []
    for i, (m, g) in enumerate(zip(demods, grid_index)):
        a = arr[i]
        a.rnti, a.n_id, a.modulation_order, a.nof_tx_layers = m.rnti, m.n_id, m.modulation_order, m.nof_tx_layers
        a.nof_rx_ports, a.start_symbol, a.nof_symbols = m.nof_rx_ports, m.start_symbol, m.nof_symbols
        a.dmrs_type, a.nof_cdm_groups_without_data, a.equalizer = (m.dmrs_type, m.nof_cdm_groups_without_data,
                                                                   m.equalizer)
        a.dmrs_symbol_mask, a.rb_start, a.nof_rb, a.grid_index = m.dmrs_symbol_mask, m.rb_start, m.nof_rb, g
        a.estimate_layout = m.estimate_layout
        a.cfo_compensated, a.numerology = m.cfo_compensated, m.numerology
        a.transform_precoding = m.transform_precoding
        a.llr_offset = off if llr_offsets is None else llr_offsets[i]
        offs.append(a.llr_offset)
        off += m.nof_llrs()
    return arr, offs, off


class PuschDemodulatorPlan:
    """srsgpu_pusch_demodulator_plan: equalization + soft demapping + descrambling of a batch of PUSCH transmissions
    from rx grids (nslots, ports, 14, nsc) and channel estimates (nslots, 4 layers, ports, 14, nsc) (uint32 bf16 pairs)
    and noise variances (ntx, 4) float32 into int8 codeword LLRs."""

    def __init__(self, ctx: Context, cfg_array, grid_nof_prb: int, grid_nof_ports: int = 4, exts=None):
        self.ctx = ctx
        h = ctypes.c_void_p()
        if exts is None:
            _check(_lib.srsgpu_pusch_demodulator_plan_create(ctx.handle, ctypes.cast(cfg_array, ctypes.c_void_p),
                                                             len(cfg_array), grid_nof_prb, grid_nof_ports,
                                                             ctypes.byref(h)))
        else:
            _check(_lib.srsgpu_pusch_demodulator_plan_create_ex(ctx.handle, ctypes.cast(cfg_array, ctypes.c_void_p),
                                                                ctypes.cast(exts, ctypes.c_void_p), len(cfg_array),
                                                                grid_nof_prb, grid_nof_ports, ctypes.byref(h)))
        self.handle = h
        self.nof_tx = len(cfg_array)

    def nof_llrs(self, tx: int) -> int:
        return int(_lib.srsgpu_pusch_demodulator_plan_nof_llrs(self.handle, tx))

    def execute(self, d_grids, d_ch_est, d_noise_var, d_llrs, stream=None, d_stats=None):
        """d_stats: optional float32 device buffer of DEMOD_STATS floats per transmission (SINR dB / EVM rows)."""
        if d_stats is None:
            _check(_lib.srsgpu_pusch_demodulator_plan_execute(self.handle, _dptr(d_grids), _dptr(d_ch_est),
                                                              _dptr(d_noise_var), _dptr(d_llrs),
                                                              _stream_handle(stream)))
        else:
            _check(_lib.srsgpu_pusch_demodulator_plan_execute_ex(self.handle, _dptr(d_grids), _dptr(d_ch_est),
                                                                 _dptr(d_noise_var), _dptr(d_llrs), _dptr(d_stats),
                                                                 _stream_handle(stream)))

    def close(self):
        if getattr(self, "handle", None):
            _lib.srsgpu_pusch_demodulator_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class PuschDemodulator:
    """GPU counterpart of srsran::pusch_demodulator::demodulate (pusch_demodulator_impl.cpp:272): demodulate() takes
    bf16 grids / channel estimates as uint16 (..., 2) arrays and returns the codeword LLRs (int8) of each
    transmission."""

    def __init__(self, ctx: Context, grid_nof_prb: int, grid_nof_ports: int = 4):
        self.ctx, self.grid_nof_prb, self.grid_nof_ports = ctx, grid_nof_prb, grid_nof_ports

    def demodulate_batch(self, grids_u16, ch_est_u16, noise_vars, demods: Sequence[PuschDemodulation],
                         grid_index: Sequence[int], with_stats: bool = False):
        """grids_u16 (S, Pg, 14, nsc, 2); ch_est_u16 (S, 4, Pg, 14, nsc, 2); noise_vars (ntx, 4). Returns the LLRs of
        each transmission and, with_stats, also the (ntx, 15, 2) statistics (SINR dB, EVM per symbol / total)."""
        dev = torch.device("cuda", self.ctx.device)
        arr, offs, total = make_pusch_demod_configs(demods, grid_index)
        exts, _keep = make_crb_mask_exts(demods, self.grid_nof_prb)
        plan = PuschDemodulatorPlan(self.ctx, arr, self.grid_nof_prb, self.grid_nof_ports, exts)
        g = torch.from_numpy(np.ascontiguousarray(grids_u16, np.uint16).view(np.int32).reshape(-1).copy()).to(dev)
        h = torch.from_numpy(np.ascontiguousarray(ch_est_u16, np.uint16).view(np.int32).reshape(-1).copy()).to(dev)
        nv = torch.from_numpy(np.ascontiguousarray(noise_vars, np.float32).reshape(-1).copy()).to(dev)
        out = torch.full((max(total, 4),), 77, dtype=torch.int8, device=dev)
        st = torch.full((max(len(demods), 1) * DEMOD_STATS,), 55.0, dtype=torch.float32, device=dev) \
            if with_stats else None
        plan.execute(g, h, nv, out, d_stats=st)
        torch.cuda.synchronize(dev)
        n = [plan.nof_llrs(i) for i in range(len(demods))]
        plan.close()
        o = out.cpu().numpy()
        llrs = [o[a:a + k] for a, k in zip(offs, n)]
        if not with_stats:
            return llrs
        return llrs, st.cpu().numpy()[:len(demods) * DEMOD_STATS].reshape(len(demods), 15, 2)


@dataclass
class PuschChannelEstimation:
    """dmrs_pusch_estimator::configuration (dmrs_pusch_estimator.h:63): pseudo-random DM-RS, contiguous CRB
    allocation (or `crb_mask`: rb_mask, one byte per grid CRB), rx ports 0..nof_rx_ports-1."""
    scrambling_id: int
    n_scid: int
    dmrs_type: int
    nof_tx_layers: int
    nof_rx_ports: int
    start_symbol: int
    nof_symbols: int
    dmrs_symbol_mask: int
    rb_start: int
    nof_rb: int
    slot_index: int
    scaling: float = 1.0
    fd_smoothing: int = CHEST_FD_FILTER
    estimate_layout: int = CE_PER_SYMBOL
    td_strategy: int = CHEST_TD_AVERAGE
    compensate_cfo: int = 0
    numerology: int = 1
    crb_mask: Optional[np.ndarray] = None
    dmrs_sequence: int = 0  # DMRS_PSEUDO_RANDOM, or DMRS_LOW_PAPR (transform precoding: scrambling_id = n_RS_ID)


DMRS_PSEUDO_RANDOM, DMRS_LOW_PAPR = 0, 1


def make_pusch_chest_configs(ests: Sequence[PuschChannelEstimation], grid_index: Sequence[int]):
    arr = (PuschChestConfig * len(ests))()
    for i, (e, g) in enumerate(zip(ests, grid_index)):
        a = arr[i]
        a.scrambling_id, a.n_scid, a.dmrs_type, a.nof_tx_layers = e.scrambling_id, e.n_scid, e.dmrs_type, e.nof_tx_layers
        a.nof_rx_ports, a.start_symbol, a.nof_symbols = e.nof_rx_ports, e.start_symbol, e.nof_symbols
        a.dmrs_symbol_mask, a.rb_start, a.nof_rb, a.slot_index = e.dmrs_symbol_mask, e.rb_start, e.nof_rb, e.slot_index
        a.estimate_layout, a.td_strategy, a.compensate_cfo = e.estimate_layout, e.td_strategy, e.compensate_cfo
        a.numerology = e.numerology
        a.fd_smoothing, a.scaling, a.grid_index = e.fd_smoothing, e.scaling, g
        a.dmrs_sequence = e.dmrs_sequence
    return arr


class PuschChannelEstimatorPlan:
    """srsgpu_pusch_chest_plan: DM-RS channel estimation of a batch of PUSCH transmissions from rx grids
    (S, Pg, 14, nsc) into estimates (S, 4, Pg, 14, nsc) (uint32 bf16 pairs), noise variances (ntx, 4) and optional
    metrics (ntx, 4, CHEST_METRICS: RSRP, EPRE, noise variance, SNR, TA seconds, CFO Hz or NaN, 0, 0)."""

    def __init__(self, ctx: Context, cfg_array, grid_nof_prb: int, grid_nof_ports: int = 4, exts=None):
        self.ctx = ctx
        h = ctypes.c_void_p()
        if exts is None:
            _check(_lib.srsgpu_pusch_chest_plan_create(ctx.handle, ctypes.cast(cfg_array, ctypes.c_void_p),
                                                       len(cfg_array), grid_nof_prb, grid_nof_ports, ctypes.byref(h)))
        else:
            _check(_lib.srsgpu_pusch_chest_plan_create_ex(ctx.handle, ctypes.cast(cfg_array, ctypes.c_void_p),
                                                          ctypes.cast(exts, ctypes.c_void_p), len(cfg_array),
                                                          grid_nof_prb, grid_nof_ports, ctypes.byref(h)))
        self.handle = h

    def execute(self, d_grids, d_ch_est, d_noise_var, d_metrics=None, stream=None):
        _check(_lib.srsgpu_pusch_chest_plan_execute(self.handle, _dptr(d_grids), _dptr(d_ch_est), _dptr(d_noise_var),
                                                    _dptr(d_metrics), _stream_handle(stream)))

    def execute_copy(self, d_grids, d_ch_est, d_noise_var, spans, d_metrics=None, stream=None):
        """execute, with the copies spans = [(src, dst)] done by extra workgroups of the same launch. Returns the
        device span list (keep it alive until the stream has run the launch)."""
        d, nbytes = span_list(spans)
        _check(_lib.srsgpu_pusch_chest_plan_execute_copy(self.handle, _dptr(d_grids), _dptr(d_ch_est),
                                                         _dptr(d_noise_var), _dptr(d_metrics), _dptr(d), len(spans),
                                                         int(nbytes.max()), _stream_handle(stream)))
        return d

    def close(self):
        if getattr(self, "handle", None):
            _lib.srsgpu_pusch_chest_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class PuschChannelEstimator:
    """GPU counterpart of srsran::dmrs_pusch_estimator::estimate (dmrs_pusch_estimator_impl.cpp:28)."""

    def __init__(self, ctx: Context, grid_nof_prb: int, grid_nof_ports: int = 4):
        self.ctx, self.grid_nof_prb, self.grid_nof_ports = ctx, grid_nof_prb, grid_nof_ports

    def estimate_batch(self, grids_u16, ests: Sequence[PuschChannelEstimation], grid_index: Sequence[int]):
        """grids_u16 (S, Pg, 14, nsc, 2) -> (estimates (S, 4, Pg, 14, nsc, 2) uint16, noise_var (ntx, 4),
        metrics (ntx, 4, CHEST_METRICS))."""
        dev = torch.device("cuda", self.ctx.device)
        exts, _keep = make_crb_mask_exts(ests, self.grid_nof_prb)
        plan = PuschChannelEstimatorPlan(self.ctx, make_pusch_chest_configs(ests, grid_index), self.grid_nof_prb,
                                         self.grid_nof_ports, exts)
        g = np.ascontiguousarray(grids_u16, np.uint16)
        S = g.shape[0]
        d_g = torch.from_numpy(g.view(np.int32).reshape(-1).copy()).to(dev)
        d_ce = torch.zeros(S * 4 * g.shape[1] * g.shape[2] * g.shape[3], dtype=torch.int32, device=dev)
        d_nv = torch.zeros(4 * len(ests), dtype=torch.float32, device=dev)
        d_m = torch.zeros(4 * CHEST_METRICS * len(ests), dtype=torch.float32, device=dev)
        plan.execute(d_g, d_ce, d_nv, d_m)
        torch.cuda.synchronize(dev)
        plan.close()
        ce = d_ce.cpu().numpy().view(np.uint16).reshape((S, 4) + g.shape[1:])
        return ce, d_nv.cpu().numpy().reshape(-1, 4), d_m.cpu().numpy().reshape(-1, 4, CHEST_METRICS)


@dataclass
class UlschDemultiplexing:
    """ulsch_demultiplex::configuration (ulsch_demultiplex.h:48) + set_csi_part2 sizes + the transmission's rnti /
    n_id (scrambling of the UCI placeholders)."""
    modulation_order: int
    nof_layers: int
    nof_prb: int
    start_symbol: int
    nof_symbols: int
    dmrs_symbol_mask: int
    dmrs_type: int
    nof_cdm_groups_without_data: int
    rnti: int
    n_id: int
    nof_harq_ack_rvd: int = 0
    nof_harq_ack_bits: int = 0
    nof_enc_harq_ack_bits: int = 0
    nof_csi_part1_bits: int = 0
    nof_enc_csi_part1_bits: int = 0
    nof_csi_part2_bits: int = 0
    nof_enc_csi_part2_bits: int = 0
    csi2_first_symbol: int = 0  # CSI Part 2 from this symbol on (the processor's set_csi_part2 point; 0: from the start)


class UlschDemuxPlan:
    """srsgpu_ulsch_demux_plan: UCI-on-PUSCH demultiplexing of a batch of codewords (int8 LLRs) into the UL-SCH,
    HARQ-ACK, CSI Part 1 and CSI Part 2 streams."""

    STREAMS = ("codeword", "sch", "harq", "csi1", "csi2")

    def __init__(self, ctx: Context, demuxes: Sequence[UlschDemultiplexing], llr_offsets: Sequence[int]):
        self.ctx = ctx
        arr = (UlschDemuxConfig * len(demuxes))()
        for i, (m, off) in enumerate(zip(demuxes, llr_offsets)):
            a = arr[i]
            for f, _ in UlschDemuxConfig._fields_:
                if hasattr(m, f):
                    setattr(a, f, getattr(m, f))
            a.llr_offset = off
        h = ctypes.c_void_p()
        # First pass sizes the output streams, the second fixes their offsets.
        _check(_lib.srsgpu_ulsch_demux_plan_create(ctx.handle, ctypes.cast(arr, ctypes.c_void_p), len(arr),
                                                   ctypes.byref(h)))
        n = [[int(_lib.srsgpu_ulsch_demux_plan_nof_llrs(h, t, k)) for k in range(5)] for t in range(len(arr))]
        _lib.srsgpu_ulsch_demux_plan_destroy(h)
        self.offsets = {k: [] for k in self.STREAMS[1:]}
        self.totals = {}
        for j, k in enumerate(self.STREAMS[1:]):
            o = 0
            for t in range(len(arr)):
                self.offsets[k].append(o)
                o += n[t][j + 1]
            self.totals[k] = o
        for t in range(len(arr)):
            arr[t].sch_offset, arr[t].harq_offset = self.offsets["sch"][t], self.offsets["harq"][t]
            arr[t].csi1_offset, arr[t].csi2_offset = self.offsets["csi1"][t], self.offsets["csi2"][t]
        h = ctypes.c_void_p()
        _check(_lib.srsgpu_ulsch_demux_plan_create(ctx.handle, ctypes.cast(arr, ctypes.c_void_p), len(arr),
                                                   ctypes.byref(h)))
        self.handle = h
        self.counts = n

    def symbol_llrs(self, tx: int, stream: str) -> np.ndarray:
        """LLRs of `stream` (codeword, sch, harq, csi1, csi2) per OFDM symbol 0..13 of transmission tx."""
        out = np.zeros(14, np.uint32)
        _check(_lib.srsgpu_ulsch_demux_plan_symbol_llrs(self.handle, tx, self.STREAMS.index(stream),
                                                        out.ctypes.data_as(ctypes.c_void_p)))
        return out

    def execute(self, d_llrs, d_sch, d_harq=None, d_csi1=None, d_csi2=None, stream=None):
        _check(_lib.srsgpu_ulsch_demux_plan_execute(self.handle, _dptr(d_llrs), _dptr(d_sch), _dptr(d_harq),
                                                    _dptr(d_csi1), _dptr(d_csi2), _stream_handle(stream)))

    def close(self):
        if getattr(self, "handle", None):
            _lib.srsgpu_ulsch_demux_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class UlschDemultiplexer:
    """GPU counterpart of srsran::ulsch_demultiplex (ulsch_demultiplex_impl.cpp:199): demultiplex_batch() takes each
    transmission's codeword LLRs and returns dicts of the sch / harq / csi1 / csi2 LLR streams."""

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def demultiplex_batch(self, codewords: Sequence[np.ndarray], demuxes: Sequence[UlschDemultiplexing]):
        dev = torch.device("cuda", self.ctx.device)
        offs, o = [], 0
        for cw in codewords:
            offs.append(o)
            o += cw.size
        plan = UlschDemuxPlan(self.ctx, demuxes, offs)
        d_in = torch.from_numpy(np.concatenate([np.asarray(c, np.int8) for c in codewords])).to(dev)
        outs = {k: torch.full((max(plan.totals[k], 4),), 99, dtype=torch.int8, device=dev) for k in plan.totals}
        plan.execute(d_in, outs["sch"], outs["harq"], outs["csi1"], outs["csi2"])
        torch.cuda.synchronize(dev)
        host = {k: v.cpu().numpy() for k, v in outs.items()}
        res = []
        for t in range(len(demuxes)):
            res.append({k: host[k][plan.offsets[k][t]: plan.offsets[k][t] + plan.counts[t][j + 1]]
                        for j, k in enumerate(("sch", "harq", "csi1", "csi2"))})
        plan.close()
        return res


class OfdmPlan:
    """srsgpu_ofdm_plan: OFDM slot modulation (inverse=True) or demodulation of nof_grids slots x nof_ports ports.
    Grids: (nof_grids, nof_ports, nsymb, 12 bw_rb) uint32 bf16 pairs; time buffer: nof_samples complex floats (as
    2 * nof_samples float32), slot of (grid, port) at sample_offset(grid, port).
    symbols=(first, count): a symbol-granularity plan of one slot (slot_indices holds one slot index) covering only
    those symbols (srsgpu_ofdm_*_symbols_plan_create; grid rows [port][symbol - first])."""

    def __init__(self, ctx: Context, inverse: bool, numerology: int, bw_rb: int, dft_size: int, scale: float,
                 center_freq_hz: float, slot_indices: Sequence[int], nof_ports: int, cp_extended: bool = False,
                 window_offset: int = 0, symbols=None):
        self.ctx, self.inverse = ctx, inverse
        cfg = OfdmConfig(numerology, bw_rb, dft_size, int(cp_extended), window_offset, scale, center_freq_hz)
        h = ctypes.c_void_p()
        if symbols is not None:
            if len(slot_indices) != 1:
                raise ValueError("a symbol-granularity plan covers one slot")
            f = (_lib.srsgpu_ofdm_modulator_symbols_plan_create if inverse
                 else _lib.srsgpu_ofdm_demodulator_symbols_plan_create)
            _check(f(ctx.handle, ctypes.byref(cfg), nof_ports, slot_indices[0], symbols[0], symbols[1],
                     ctypes.byref(h)))
        else:
            slots = (ctypes.c_uint32 * max(len(slot_indices), 1))(*slot_indices)
            f = _lib.srsgpu_ofdm_modulator_plan_create if inverse else _lib.srsgpu_ofdm_demodulator_plan_create
            _check(f(ctx.handle, ctypes.byref(cfg), len(slot_indices), nof_ports,
                     ctypes.cast(slots, ctypes.c_void_p), ctypes.byref(h)))
        self.handle = h
        self.nof_grids, self.nof_ports = len(slot_indices), nof_ports
        self.nsymb, self.nsc = (12 if cp_extended else 14), 12 * bw_rb
        if symbols is not None:
            self.nsymb = symbols[1]
        self.nof_samples = int(_lib.srsgpu_ofdm_plan_nof_samples(h))
        self.grid_words = int(_lib.srsgpu_ofdm_plan_nof_grid_words(h))

    @classmethod
    def concat(cls, members: Sequence["OfdmPlan"]) -> "OfdmPlan":
        """srsgpu_ofdm_plan_concat: one plan running the members' jobs (a sector group): member i's grid words and time
        samples follow member i-1's."""
        arr = (ctypes.c_void_p * len(members))(*[m.handle for m in members])
        h = ctypes.c_void_p()
        _check(_lib.srsgpu_ofdm_plan_concat(members[0].ctx.handle, ctypes.cast(arr, ctypes.c_void_p), len(members),
                                             ctypes.byref(h)))
        self = cls.__new__(cls)
        self.ctx, self.inverse, self.handle = members[0].ctx, members[0].inverse, h
        self.nof_grids = sum(m.nof_grids for m in members)
        self.nof_ports, self.nsymb, self.nsc = members[0].nof_ports, members[0].nsymb, members[0].nsc
        self.nof_samples = int(_lib.srsgpu_ofdm_plan_nof_samples(h))
        self.grid_words = int(_lib.srsgpu_ofdm_plan_nof_grid_words(h))
        return self

    def sample_offset(self, grid: int, port: int) -> int:
        return int(_lib.srsgpu_ofdm_plan_sample_offset(self.handle, grid, port))

    OFDM_JOB = np.dtype([("grid_offset", "<u4"), ("sample_offset", "<u4"), ("cp_len", "<u4"), ("reserved", "<u4"),
                         ("coef_re", "<f4"), ("coef_im", "<f4")])

    def jobs(self) -> np.ndarray:
        """srsgpu_ofdm_plan_get_jobs: the plan's (grid, port, symbol) jobs as a structured array (OFDM_JOB)."""
        n = ctypes.c_uint32()
        _check(_lib.srsgpu_ofdm_plan_get_jobs(self.handle, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, self.OFDM_JOB)
        _check(_lib.srsgpu_ofdm_plan_get_jobs(self.handle, out.ctypes.data, n.value, ctypes.byref(n)))
        return out

    def execute_jobs(self, d_jobs, nof_jobs: int, d_in, d_out, stream=None):
        """srsgpu_ofdm_jobs_execute: a caller-assembled job list with this plan's launch parameters."""
        _check(_lib.srsgpu_ofdm_jobs_execute(self.handle, _dptr(d_jobs), nof_jobs, _dptr(d_in), _dptr(d_out),
                                             _stream_handle(stream)))

    OFDM_DIRECT_JOB = np.dtype([("grid", "<u8"), ("samples", "<u8"), ("cp_len", "<u4"), ("coef_re", "<f4"),
                                ("coef_im", "<f4"), ("reserved", "<u4"), ("grid_copy", "<u8")])

    def direct_jobs(self, d_grid, d_samples) -> np.ndarray:
        """The plan's jobs as srsgpu_ofdm_direct_job (OFDM_DIRECT_JOB) over the given grid and sample buffers."""
        j = self.jobs()
        out = np.zeros(len(j), self.OFDM_DIRECT_JOB)
        out["grid"] = _dptr(d_grid) + 4 * j["grid_offset"].astype(np.uint64)
        out["samples"] = _dptr(d_samples) + 8 * j["sample_offset"].astype(np.uint64)
        out["cp_len"], out["coef_re"], out["coef_im"] = j["cp_len"], j["coef_re"], j["coef_im"]
        return out

    def execute_jobs_direct(self, d_jobs, nof_jobs: int, stream=None):
        """srsgpu_ofdm_jobs_execute_direct: direct-address jobs with this plan's launch parameters."""
        _check(_lib.srsgpu_ofdm_jobs_execute_direct(self.handle, _dptr(d_jobs), nof_jobs, _stream_handle(stream)))

    def execute(self, d_in, d_out, stream=None):
        f = _lib.srsgpu_ofdm_modulator_plan_execute if self.inverse else _lib.srsgpu_ofdm_demodulator_plan_execute
        _check(f(self.handle, _dptr(d_in), _dptr(d_out), _stream_handle(stream)))

    def execute_twin(self, d_grid, d_twin, d_samples, stream=None):
        """srsgpu_ofdm_modulator_plan_execute_twin: every RE from d_twin unless it holds 0xffffffff, else from d_grid."""
        _check(_lib.srsgpu_ofdm_modulator_plan_execute_twin(self.handle, _dptr(d_grid), _dptr(d_twin), _dptr(d_samples),
                                                            _stream_handle(stream)))

    def close(self):
        if getattr(self, "handle", None):
            _lib.srsgpu_ofdm_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class OfdmSlotModulator:
    """GPU counterpart of srsran::ofdm_slot_modulator (ofdm_modulator_impl.cpp:115): modulate(grid, slot) takes a
    (nof_ports, nsymb, 12 bw_rb, 2) bf16 grid and returns (nof_ports, slot_size) complex64 samples."""

    def __init__(self, ctx: Context, numerology, bw_rb, dft_size, scale, center_freq_hz, cp_extended=False):
        self.ctx = ctx
        self.args = (numerology, bw_rb, dft_size, scale, center_freq_hz)
        self.cp_extended = cp_extended

    def modulate(self, grid_u16: np.ndarray, slot_index: int) -> np.ndarray:
        P = grid_u16.shape[0]
        plan = OfdmPlan(self.ctx, True, *self.args, [slot_index], P, self.cp_extended)
        dev = torch.device("cuda", self.ctx.device)
        g = np.ascontiguousarray(grid_u16, np.uint16).view(np.int32).reshape(-1)
        d_grid = torch.from_numpy(g.copy()).to(dev)
        d_out = torch.zeros(2 * plan.nof_samples, dtype=torch.float32, device=dev)
        plan.execute(d_grid, d_out)
        torch.cuda.synchronize(dev)
        plan.close()
        return d_out.cpu().numpy().view(np.complex64).reshape(P, -1)


class OfdmSlotDemodulator:
    """GPU counterpart of srsran::ofdm_slot_demodulator (ofdm_demodulator_impl.cpp:154): demodulate(samples, slot)
    takes (nof_ports, slot_size) complex samples and returns the (nof_ports, nsymb, 12 bw_rb, 2) bf16 grid."""

    def __init__(self, ctx: Context, numerology, bw_rb, dft_size, scale, center_freq_hz, cp_extended=False,
                 window_offset=0):
        self.ctx = ctx
        self.args = (numerology, bw_rb, dft_size, scale, center_freq_hz)
        self.cp_extended, self.window_offset = cp_extended, window_offset

    def demodulate(self, samples: np.ndarray, slot_index: int) -> np.ndarray:
        P = samples.shape[0]
        plan = OfdmPlan(self.ctx, False, *self.args, [slot_index], P, self.cp_extended, self.window_offset)
        dev = torch.device("cuda", self.ctx.device)
        x = np.ascontiguousarray(samples, np.complex64).view(np.float32).reshape(-1)
        d_in = torch.from_numpy(x.copy()).to(dev)
        d_grid = torch.zeros(P * plan.nsymb * plan.nsc, dtype=torch.int32, device=dev)
        plan.execute(d_in, d_grid)
        torch.cuda.synchronize(dev)
        plan.close()
        return d_grid.cpu().numpy().view(np.uint16).reshape(P, plan.nsymb, plan.nsc, 2)


@dataclass
class PuschTransportBlock:
    """pusch_decoder::configuration (pusch_decoder.h:55) + the TB geometry of one transport block."""
    tbs_bytes: int
    base_graph: int
    rv: int
    modulation_order: int
    nof_layers: int
    nof_ch_symbols: int
    Nref: int = 0
    new_data: bool = True
    use_early_stop: bool = True
    nof_ldpc_iterations: int = 6
    scaling_factor: float = 0.8


def make_pusch_tb_configs(tbs: Sequence[PuschTransportBlock], nof_cbs: Sequence[int], cb_lengths: Sequence[int]):
    """Contiguous layout: codeword LLRs, HARQ buffers (C * N per TB), codeblock slots, TB bytes.
    nof_cbs[i] / cb_lengths[i] (N_short * Z) come from the segmentation (srsgpu.sch)."""
    arr = (PuschTbConfig * len(tbs))()
    lo = ho = co = to = 0
    for i, t in enumerate(tbs):
        a = arr[i]
        a.base_graph, a.rv, a.modulation_order, a.nof_layers = t.base_graph, t.rv, t.modulation_order, t.nof_layers
        a.new_data, a.use_early_stop, a.max_iterations = int(t.new_data), int(t.use_early_stop), t.nof_ldpc_iterations
        a.scaling_factor, a.tbs_bytes, a.nof_ch_symbols, a.Nref = t.scaling_factor, t.tbs_bytes, t.nof_ch_symbols, t.Nref
        a.llr_offset, a.harq_offset, a.cb_offset, a.tb_offset = lo, ho, co, to
        lo += t.nof_ch_symbols * t.modulation_order
        ho += nof_cbs[i] * cb_lengths[i]
        co += nof_cbs[i]
        to += t.tbs_bytes
    return arr, lo, ho, co, to


class PuschDecoderPlan:
    """srsgpu_pusch_decoder_plan (TB level)."""

    def __init__(self, ctx: Context, impl: int, cfg_array):
        self.ctx = ctx
        h = ctypes.c_void_p()
        _check(_lib.srsgpu_pusch_decoder_plan_create(ctx.handle, impl, ctypes.cast(cfg_array, ctypes.c_void_p),
                                                     len(cfg_array), ctypes.byref(h)))
        self.handle = h
        self.nof_tbs = len(cfg_array)
        self.nof_codeblocks = int(_lib.srsgpu_pusch_decoder_plan_nof_codeblocks(h))
        self.decoder_input_llrs = int(_lib.srsgpu_pusch_decoder_plan_decoder_input_llrs(h))

    def execute(self, d_llrs, d_harq, d_cb_crc_ok, d_cb_msgs, d_cb_iters, d_tbs, d_tb_crc_ok, stream=None):
        _check(_lib.srsgpu_pusch_decoder_plan_execute(self.handle, _dptr(d_llrs), _dptr(d_harq), _dptr(d_cb_crc_ok),
                                                      _dptr(d_cb_msgs), _dptr(d_cb_iters), _dptr(d_tbs),
                                                      _dptr(d_tb_crc_ok), _stream_handle(stream)))

    def execute_arena(self, d_llrs, d_harq_cbs, d_cb_crc_ok, d_cb_msgs, d_cb_iters, d_tbs, d_tb_crc_ok, stream=None):
        """As execute, with codeblock c's HARQ soft buffer at the device address d_harq_cbs[c] (an int64 tensor of one
        pointer per codeblock, e.g. slots of a persistent arena) instead of in a contiguous batch buffer."""
        _check(_lib.srsgpu_pusch_decoder_plan_execute_arena(self.handle, _dptr(d_llrs), _dptr(d_harq_cbs),
                                                            _dptr(d_cb_crc_ok), _dptr(d_cb_msgs), _dptr(d_cb_iters),
                                                            _dptr(d_tbs), _dptr(d_tb_crc_ok), _stream_handle(stream)))

    def assemble(self, d_cb_crc_ok, d_cb_msgs, d_tbs, d_tb_crc_ok, stream=None):
        """TB stage only, from codeblock messages / flags decoded elsewhere (codeblock-sharded decoding)."""
        _check(_lib.srsgpu_pusch_decoder_plan_assemble(self.handle, _dptr(d_cb_crc_ok), _dptr(d_cb_msgs), _dptr(d_tbs),
                                                       _dptr(d_tb_crc_ok), _stream_handle(stream)))

    def enable_timing(self, enable=True, decode_only=False):
        """Stage events on every execute: all three stages, or (decode_only) just around the LDPC decoding."""
        _check(_lib.srsgpu_pusch_decoder_plan_enable_timing(self.handle, (2 if decode_only else 1) if enable else 0))

    def stage_times(self):
        """([ms dematch, ms decode, ms TB stage], number of executes) accumulated since the previous call."""
        return _stage_times("srsgpu_pusch_decoder_plan", self.handle, 3)

    def close(self):
        if getattr(self, "handle", None):
            _lib.srsgpu_pusch_decoder_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class PuschDecoder:
    """GPU counterpart of srsran::pusch_decoder with a device-resident HARQ context (one per set of TBs)."""

    def __init__(self, ctx: Context, dec_type: str = "auto"):
        if dec_type not in IMPL_BY_NAME:
            raise SrsGpuError(f"invalid decoder type '{dec_type}'")
        self.ctx = ctx
        self.impl = IMPL_BY_NAME[dec_type]
        self.harq = None

    def decode_batch(self, llrs_list, tbs: Sequence[PuschTransportBlock]):
        """Returns (tb_crc_ok list, TB byte arrays, per-TB lists of CB iteration counts). The HARQ context is kept
        between calls (retransmissions: same TBs, new_data False)."""
        from . import sch
        nof_cbs, cb_len = [], []
        for t in tbs:
            seg = sch.segment(t.tbs_bytes * 8, t.base_graph, t.modulation_order, t.nof_layers, t.nof_ch_symbols)
            nof_cbs.append(seg.nof_segments)
            cb_len.append((66 if t.base_graph == 1 else 50) * seg.lifting_size)
        arr, nllr, nharq, ncb, ntb = make_pusch_tb_configs(tbs, nof_cbs, cb_len)
        dev = torch.device("cuda", self.ctx.device)
        if self.harq is None or self.harq[0].numel() != nharq:
            self.harq = (torch.zeros(nharq, dtype=torch.int8, device=dev),
                         torch.zeros(ncb, dtype=torch.uint8, device=dev),
                         torch.zeros(ncb * CB_MSG_STRIDE, dtype=torch.uint8, device=dev))
        d_harq, d_crc, d_msgs = self.harq
        d_llrs = torch.from_numpy(np.concatenate([np.asarray(x, np.int8) for x in llrs_list])).to(dev)
        assert d_llrs.numel() == nllr
        d_iters = torch.zeros(ncb, dtype=torch.int32, device=dev)
        d_tbs = torch.zeros(max(ntb, 1), dtype=torch.uint8, device=dev)
        d_tb_ok = torch.zeros(len(tbs), dtype=torch.uint8, device=dev)
        plan = PuschDecoderPlan(self.ctx, self.impl, arr)
        plan.execute(d_llrs, d_harq, d_crc, d_msgs, d_iters, d_tbs, d_tb_ok)
        torch.cuda.synchronize(dev)
        plan.close()
        ok = d_tb_ok.cpu().numpy()
        tb_bytes = d_tbs.cpu().numpy()
        iters = d_iters.cpu().numpy()
        out_tbs, out_iters = [], []
        off = co = 0
        for i, t in enumerate(tbs):
            out_tbs.append(tb_bytes[off: off + t.tbs_bytes].copy())
            out_iters.append(iters[co: co + nof_cbs[i]].tolist())
            off += t.tbs_bytes
            co += nof_cbs[i]
        return [bool(x) for x in ok], out_tbs, out_iters
