"""Test-side loaders for the CPU oracle (oracle/liboracle.so) and the reference build (oracle/_ref/libsrsref.so).

TEST INFRASTRUCTURE ONLY: these are the checkers; the product (srsran-5g_amd/) never imports this module.
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libsrsref.so")

CRC24A, CRC24B, CRC24C, CRC16, CRC11, CRC6 = range(6)
CRC_LEN = {CRC24A: 24, CRC24B: 24, CRC24C: 24, CRC16: 16, CRC11: 11, CRC6: 6}
LIFTING_SIZES = [2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 20, 22, 24, 26, 28, 30, 32, 36, 40, 44, 48,
                 52, 56, 60, 64, 72, 80, 88, 96, 104, 112, 120, 128, 144, 160, 176, 192, 208, 224, 240, 256, 288, 320,
                 352, 384]
BG_K = {1: 22, 2: 10}
BG_N_SHORT = {1: 66, 2: 50}

_P = ctypes.c_void_p


def _ptr(a):
    return a.ctypes.data_as(_P)


def _setup(lib, prefix):
    f = getattr(lib, prefix + "crc_bits")
    f.restype = ctypes.c_uint
    f.argtypes = [ctypes.c_int, _P, ctypes.c_uint]
    f = getattr(lib, prefix + "crc_bytes")
    f.restype = ctypes.c_uint
    f.argtypes = [ctypes.c_int, _P, ctypes.c_uint]
    f = getattr(lib, prefix + "ldpc_decode")
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int] * 7 + [ctypes.c_float, _P, ctypes.c_uint, _P]


class _Lib:
    def __init__(self, path, prefix):
        self.lib = ctypes.CDLL(path)
        self.prefix = prefix
        _setup(self.lib, prefix)

    def _f(self, name):
        return getattr(self.lib, self.prefix + name)

    def crc_bits(self, poly, bits):
        bits = np.ascontiguousarray(bits, dtype=np.uint8)
        return int(self._f("crc_bits")(poly, _ptr(bits), bits.size))

    def crc_bytes(self, poly, data):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        return int(self._f("crc_bytes")(poly, _ptr(data), data.size))

    def ldpc_decode(self, mode, bg, Z, llr, nof_crc_bits=16, nof_filler=0, crc_poly=-1, max_iter=6, scaling=0.8,
                    out_init=None):
        llr = np.ascontiguousarray(llr, dtype=np.int8)
        K = BG_K[bg]
        out = np.zeros(K * Z, np.uint8) if out_init is None else np.array(out_init, dtype=np.uint8)
        r = self._f("ldpc_decode")(mode, bg, Z, nof_crc_bits, nof_filler, crc_poly, max_iter, scaling, _ptr(llr),
                                  llr.size, _ptr(out))
        return r, out

    def pdsch_modulate(self, cfg, weights, cw_packed, nof_bits, grid_nof_prb, grid=None):
        """PDSCH modulator (ref_pdsch_modulate / orc_pdsch_modulate): returns the grid as uint16 bf16 bit patterns,
        shape (nof_ports, 14, 12 * grid_nof_prb, 2). `cfg` is a PdschModConfig-like mapping (see PDSCH_MOD_KEYS)."""
        f = self._f("pdsch_modulate")
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_int] * 11 + [ctypes.c_uint, ctypes.c_int, ctypes.c_int, ctypes.c_float, _P, _P,
                                            ctypes.c_int, ctypes.c_int, _P]
        w = np.ascontiguousarray(weights, dtype=np.complex64).view(np.float32)
        cw = np.ascontiguousarray(cw_packed, dtype=np.uint8)
        if grid is None:
            grid = np.zeros((cfg["nof_ports"], 14, 12 * grid_nof_prb, 2), np.uint16)
        r = f(*[int(cfg[k]) for k in PDSCH_MOD_KEYS[:11]], ctypes.c_uint(int(cfg["dmrs_symbol_mask"])),
              int(cfg["dmrs_type2"]), int(cfg["nof_cdm_groups_without_data"]), float(cfg["scaling"]), _ptr(w),
              _ptr(cw), int(nof_bits), int(grid_nof_prb), _ptr(grid))
        assert r == 0, r
        return grid


def _general_args(cfg, grid_nof_prb):
    res = cfg["reserved"]
    res_crb = (np.concatenate([np.asarray(r[0], np.uint8)[:grid_nof_prb] for r in res]) if res
               else np.zeros(1, np.uint8))
    res_re = np.array([r[1] for r in res] or [0], np.uint16)
    res_sym = np.array([r[2] for r in res] or [0], np.uint16)
    pw = (np.ascontiguousarray(cfg["prg_weights"], np.complex64).view(np.float32) if cfg["prg_size"]
          else np.zeros(2, np.float32))
    nprg = cfg["prg_weights"].shape[0] if cfg["prg_size"] else 0
    return res_crb, res_re, res_sym, pw, nprg


def pdsch_modulate_general(lib, cfg, weights, cw_packed, nof_bits, grid_nof_prb, crb_mask=None, grid=None):
    """orc_pdsch_modulate_ex (crb_mask given) / ref_pdsch_modulate_ex (VRB mask + interleaving of cfg): returns
    (grid (P, 14, nsc, 2) uint16, CRB mask uint8 (the reference's get_crb_mask, or crb_mask))."""
    w = np.ascontiguousarray(weights, dtype=np.complex64).view(np.float32)
    cw = np.ascontiguousarray(cw_packed, dtype=np.uint8)
    res_crb, res_re, res_sym, pw, nprg = _general_args(cfg, grid_nof_prb)
    if grid is None:
        grid = np.zeros((cfg["nof_ports"], 14, 12 * grid_nof_prb, 2), np.uint16)
    head = [int(cfg[k]) for k in ("rnti", "n_id", "qm", "nof_layers", "nof_ports", "bwp_start_rb", "bwp_size_rb")]
    mid = [int(cfg["start_symbol"]), int(cfg["nof_symbols"]), ctypes.c_uint(int(cfg["dmrs_symbol_mask"])),
           int(cfg["dmrs_type2"]), int(cfg["nof_cdm_groups_without_data"]), ctypes.c_float(float(cfg["scaling"])),
           _ptr(w), len(cfg["reserved"]), _ptr(res_crb), _ptr(res_re), _ptr(res_sym), int(cfg["prg_size"]), nprg,
           _ptr(pw), _ptr(cw), int(nof_bits), int(grid_nof_prb), _ptr(grid)]
    if crb_mask is not None:
        crb = np.ascontiguousarray(crb_mask, np.uint8)
        f = lib.orc_pdsch_modulate_ex
        f.restype = ctypes.c_int
        r = f(*head, _ptr(crb), *mid)
    else:
        vrb = np.ascontiguousarray(cfg["vrb_mask"], np.uint8)
        crb = np.zeros(grid_nof_prb, np.uint8)
        f = lib.ref_pdsch_modulate_ex
        f.restype = ctypes.c_int
        r = f(*head, _ptr(vrb), vrb.size, int(cfg["interleave"]), *mid, _ptr(crb))
    assert r == 0, r
    return grid, crb


PDSCH_MOD_KEYS = ["rnti", "n_id", "qm", "nof_layers", "nof_ports", "bwp_start_rb", "bwp_size_rb", "rb_start", "nof_rb",
                  "start_symbol", "nof_symbols", "dmrs_symbol_mask", "dmrs_type2", "nof_cdm_groups_without_data",
                  "scaling"]


def pdsch_mod_nof_re(cfg):
    """Data REs of a PDSCH modulator configuration (DM-RS REs of the DM-RS symbols excluded)."""
    if cfg["dmrs_type2"]:
        dm = 4 * cfg["nof_cdm_groups_without_data"]
    else:
        dm = 6 * cfg["nof_cdm_groups_without_data"]
    n = 0
    for l in range(cfg["start_symbol"], cfg["start_symbol"] + cfg["nof_symbols"]):
        n += (12 - dm if (cfg["dmrs_symbol_mask"] >> l) & 1 else 12) * cfg["nof_rb"]
    return n


class Oracle(_Lib):
    def __init__(self, path=ORACLE_SO):
        super().__init__(path, "orc_")

    def ldpc_encode(self, bg, Z, msg):
        msg = np.ascontiguousarray(msg, dtype=np.uint8)
        cb = np.zeros(BG_N_SHORT[bg] * Z, np.uint8)
        r = self.lib.orc_ldpc_encode(bg, Z, _ptr(msg), _ptr(cb))
        assert r == 0, r
        return cb

    def rate_match(self, bg, Z, rv, qm, Nref, nof_filler, cb, E):
        cb = np.ascontiguousarray(cb, dtype=np.uint8)
        out = np.zeros(E, np.uint8)
        r = self.lib.orc_rate_match(bg, Z, rv, qm, ctypes.c_uint(Nref), ctypes.c_uint(nof_filler), _ptr(cb),
                                    ctypes.c_uint(E), _ptr(out))
        assert r == 0, r
        return out

    def rate_dematch(self, mode, bg, Z, rv, qm, Nref, nof_filler, new_data, llr, buf):
        llr = np.ascontiguousarray(llr, dtype=np.int8)
        buf = np.array(buf, dtype=np.int8)
        r = self.lib.orc_rate_dematch(mode, bg, Z, rv, qm, ctypes.c_uint(Nref), ctypes.c_uint(nof_filler),
                                      int(new_data), _ptr(llr), ctypes.c_uint(llr.size), _ptr(buf))
        assert r == 0, r
        return buf


class Reference(_Lib):
    """The srsRAN reference itself, built from its own sources (oracle/build_ref.sh)."""

    GENERIC, AVX2, AVX512 = 0, 1, 2

    def __init__(self, path=REF_SO):
        super().__init__(path, "ref_")

    def has_avx512(self):
        return bool(self.lib.ref_cpu_has_avx512())

    def demodulate_soft(self, qm, symbols, noise_vars):
        """demodulation_mapper_impl::demodulate_soft: complex symbols + noise variances -> int8 LLRs."""
        x = np.ascontiguousarray(symbols, dtype=np.complex64)
        nv = np.ascontiguousarray(noise_vars, dtype=np.float32)
        out = np.zeros(x.size * qm, np.int8)
        f = self.lib.ref_demodulate_soft
        f.restype = None
        f.argtypes = [ctypes.c_int, _P, _P, ctypes.c_int, _P]
        f(qm, _ptr(x), _ptr(nv), x.size, _ptr(out))
        return out

    def pusch_demodulate(self, cfg, grid_u16, ch_est_u16, noise_var, grid_nof_prb, mmse=False):
        """pusch_demodulator_impl::demodulate of one transmission (see ref_pusch_demodulate): codeword LLRs."""
        g = np.ascontiguousarray(grid_u16, dtype=np.uint16)
        h = np.ascontiguousarray(ch_est_u16, dtype=np.uint16)
        nv = np.ascontiguousarray(noise_var, dtype=np.float32)
        cap = 12 * cfg["nof_rb"] * 14 * cfg["nof_layers"] * cfg["qm"]
        out = np.zeros(cap, np.int8)
        f = self.lib.ref_pusch_demodulate
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_int] * 7 + [ctypes.c_uint] + [ctypes.c_int] * 6 + [_P] * 4 + [ctypes.c_int]
        n = f(cfg["rnti"], cfg["n_id"], cfg["qm"], cfg["nof_layers"], cfg["nof_rx_ports"], cfg["start_symbol"],
              cfg["nof_symbols"], cfg["dmrs_symbol_mask"], cfg["dmrs_type2"], cfg["nof_cdm_groups_without_data"],
              cfg["rb_start"], cfg["nof_rb"], grid_nof_prb, int(mmse), _ptr(g), _ptr(h), _ptr(nv), _ptr(out), cap)
        return out[:n]

    def pusch_demodulate_ex(self, cfg, grid_u16, ch_est_u16, noise_var, grid_nof_prb, mmse=False, crb_mask=None,
                            transform_precoding=False):
        """ref_pusch_demodulate_ex: (codeword LLRs, stats (15, 2) float32 = per-symbol / end (SINR dB, EVM), NaN when
        absent) with a general CRB mask, transform precoding, the EVM calculator and the post-equalization SINR."""
        g = np.ascontiguousarray(grid_u16, dtype=np.uint16)
        h = np.ascontiguousarray(ch_est_u16, dtype=np.uint16)
        nv = np.ascontiguousarray(noise_var, dtype=np.float32)
        cap = 12 * grid_nof_prb * 14 * cfg["nof_layers"] * cfg["qm"]
        out = np.zeros(cap, np.int8)
        stats = np.zeros((15, 2), np.float32)
        m = None if crb_mask is None else np.ascontiguousarray(np.asarray(crb_mask, np.uint8)[:grid_nof_prb])
        f = self.lib.ref_pusch_demodulate_ex
        f.restype = ctypes.c_int
        f.argtypes = ([ctypes.c_int] * 7 + [ctypes.c_uint] + [ctypes.c_int] * 4 + [_P] + [ctypes.c_int] * 3 + [_P] * 4
                      + [ctypes.c_int, _P])
        n = f(cfg["rnti"], cfg["n_id"], cfg["qm"], cfg["nof_layers"], cfg["nof_rx_ports"], cfg["start_symbol"],
              cfg["nof_symbols"], cfg["dmrs_symbol_mask"], cfg["dmrs_type2"], cfg["nof_cdm_groups_without_data"],
              cfg["rb_start"], cfg["nof_rb"], None if m is None else _ptr(m), int(transform_precoding), grid_nof_prb,
              int(mmse), _ptr(g), _ptr(h), _ptr(nv), _ptr(out), cap, _ptr(stats))
        return out[:n], stats

    def ulsch_demux(self, cfg, llrs, c_init, csi2_bits=0, csi2_enc_bits=0, block_size=1 << 20, csi2_after_csi1=False):
        """ulsch_demultiplex_impl fed the codeword in blocks: dict sch / harq / csi1 / csi2 of int8 LLRs.
        csi2_after_csi1: set_csi_part2 when the CSI Part 1 buffer ends (the PUSCH processor's timing), else before the
        first symbol."""
        x = np.ascontiguousarray(llrs, dtype=np.int8)
        cap = x.size + 64
        outs = [np.zeros(cap, np.int8) for _ in range(4)]
        counts = np.zeros(4, np.int32)
        f = self.lib.ref_ulsch_demux_ex
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_int] * 5 + [ctypes.c_uint] + [ctypes.c_int] * 9 + [ctypes.c_uint, _P, ctypes.c_int,
                                                                                   ctypes.c_int] + [_P] * 4 + \
            [ctypes.c_int, _P, ctypes.c_int]
        f(cfg["qm"], cfg["nof_layers"], cfg["nof_prb"], cfg["start_symbol"], cfg["nof_symbols"],
          cfg["dmrs_symbol_mask"], cfg["dmrs_type2"], cfg["nof_cdm_groups_without_data"], cfg["nof_harq_ack_rvd"],
          cfg["nof_harq_ack_bits"], cfg["nof_enc_harq_ack_bits"], cfg["nof_csi_part1_bits"],
          cfg["nof_enc_csi_part1_bits"], csi2_bits, csi2_enc_bits, c_init, _ptr(x), x.size, block_size,
          *[_ptr(o) for o in outs], cap, _ptr(counts), int(csi2_after_csi1))
        return {k: o[:n] for k, o, n in zip(("sch", "harq", "csi1", "csi2"), outs, counts)}

    def low_papr(self, u, v, m):
        """low_papr_sequence_generator_impl::generate(sequence of m, u, v, 0, 1): complex64 (m,)."""
        out = np.zeros(m, np.complex64)
        f = self.lib.ref_low_papr_generate
        f.restype = None
        f.argtypes = [ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, _P]
        f(u, v, m, _ptr(out))
        return out

    def pusch_chest(self, cfg, grid_u16, grid_nof_prb, fd=2, td=0, compensate_cfo=False, numerology=1,
                    crb_mask=None, low_papr_id=-1):
        """dmrs_pusch_estimator_impl::estimate of one single-layer transmission: (ch_est (P, 14, nsc, 2) bf16,
        noise_var, rsrp, epre, ta_s, cfo_hz) per port. crb_mask (one byte per grid CRB) replaces the contiguous
        allocation as configuration::rb_mask."""
        g = np.ascontiguousarray(grid_u16, dtype=np.uint16)
        P = cfg["nof_rx_ports"]
        ce = np.zeros((P, 14, 12 * grid_nof_prb, 2), np.uint16)
        outs = [np.zeros(P, np.float32) for _ in range(5)]
        m = None if crb_mask is None else np.ascontiguousarray(np.asarray(crb_mask, np.uint8)[:grid_nof_prb])
        f = self.lib.ref_pusch_chest_mask
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_int] * 7 + [ctypes.c_float, ctypes.c_uint] + [ctypes.c_int] * 4 + [_P] + \
            [ctypes.c_int] * 5 + [_P] * 7
        f(numerology, int(low_papr_id), cfg["slot"], cfg["scrambling_id"], cfg["n_scid"], cfg["dmrs_type2"], 1, cfg["scaling"],
          cfg["dmrs_symbol_mask"], cfg["start_symbol"], cfg["nof_symbols"], cfg["rb_start"], cfg["nof_rb"],
          None if m is None else _ptr(m), grid_nof_prb, P, fd, td, int(compensate_cfo), _ptr(g), _ptr(ce),
          *[_ptr(o) for o in outs])
        return (ce,) + tuple(outs)

    def dmrs_pdsch_map(self, cfg, weights, grid_nof_prb, numerology=1, crb_mask=None):
        """dmrs_pdsch_processor_impl::map into a zeroed grid: (P, 14, nsc, 2) bf16 bit patterns. crb_mask (one byte
        per grid CRB) replaces the contiguous rb_start / nof_rb allocation as config_t::rb_mask."""
        w = np.ascontiguousarray(weights, dtype=np.complex64).view(np.float32)
        P = cfg["nof_ports"]
        grid = np.zeros((P, 14, 12 * grid_nof_prb, 2), np.uint16)
        m = None if crb_mask is None else np.ascontiguousarray(np.asarray(crb_mask, np.uint8)[:grid_nof_prb])
        f = self.lib.ref_dmrs_pdsch_map_mask
        f.restype = ctypes.c_int
        f.argtypes = ([ctypes.c_int] * 7 + [ctypes.c_uint] + [ctypes.c_int] * 3 + [ctypes.c_float, _P, _P,
                                                                                  ctypes.c_int, _P])
        f(numerology, cfg["slot"], cfg["scrambling_id"], cfg["n_scid"], cfg["dmrs_type2"], cfg["nof_layers"], P,
          cfg["dmrs_symbol_mask"], cfg["reference_point_k_rb"], cfg["rb_start"], cfg["nof_rb"], cfg["amplitude"],
          _ptr(w), None if m is None else _ptr(m), grid_nof_prb, _ptr(grid))
        return grid

    def ofdm_slot_size(self, numerology, bw_rb, dft_size, extended, slot):
        return int(self.lib.ref_ofdm_slot_size(numerology, bw_rb, dft_size, int(extended), slot))

    def ofdm_modulate(self, grid_u16, numerology, bw_rb, dft_size, extended, scale, center_freq_hz, slot):
        """ofdm_slot_modulator_impl::modulate of every port: (P, slot_size) complex64."""
        g = np.ascontiguousarray(grid_u16, dtype=np.uint16)
        P = g.shape[0]
        n = self.ofdm_slot_size(numerology, bw_rb, dft_size, extended, slot)
        out = np.zeros((P, n), np.complex64)
        f = self.lib.ref_ofdm_modulate
        f.argtypes = [ctypes.c_int] * 4 + [ctypes.c_float, ctypes.c_double, ctypes.c_int, ctypes.c_int, _P, _P]
        f(numerology, bw_rb, dft_size, int(extended), scale, center_freq_hz, slot, P, _ptr(g), _ptr(out))
        return out

    def ofdm_demodulate(self, samples, numerology, bw_rb, dft_size, extended, scale, center_freq_hz, slot,
                        window_offset=0):
        """ofdm_slot_demodulator_impl::demodulate of every port: (P, nsymb, 12 bw_rb, 2) bf16 bit patterns."""
        x = np.ascontiguousarray(samples, dtype=np.complex64)
        P = x.shape[0]
        ns = 12 if extended else 14
        grid = np.zeros((P, ns, 12 * bw_rb, 2), np.uint16)
        f = self.lib.ref_ofdm_demodulate
        f.argtypes = [ctypes.c_int] * 4 + [ctypes.c_float, ctypes.c_double] + [ctypes.c_int] * 3 + [_P, _P]
        f(numerology, bw_rb, dft_size, int(extended), scale, center_freq_hz, window_offset, slot, P, _ptr(x),
          _ptr(grid))
        return grid

    def ldpc_encode(self, bg, Z, msg, impl=0):
        msg = np.ascontiguousarray(msg, dtype=np.uint8)
        cb = np.zeros(BG_N_SHORT[bg] * Z, np.uint8)
        self.lib.ref_ldpc_encode(impl, bg, Z, _ptr(msg), _ptr(cb))
        return cb

    def rate_match(self, bg, Z, rv, qm, Nref, nof_filler, msg, E):
        msg = np.ascontiguousarray(msg, dtype=np.uint8)
        out = np.zeros(E, np.uint8)
        self.lib.ref_rate_match(bg, Z, rv, qm, ctypes.c_uint(Nref), ctypes.c_uint(nof_filler), _ptr(msg),
                                ctypes.c_uint(E), _ptr(out))
        return out

    def rate_dematch(self, impl, bg, Z, rv, qm, Nref, nof_filler, new_data, llr, buf):
        llr = np.ascontiguousarray(llr, dtype=np.int8)
        buf = np.array(buf, dtype=np.int8)
        self.lib.ref_rate_dematch(impl, bg, Z, rv, qm, ctypes.c_uint(Nref), ctypes.c_uint(nof_filler), int(new_data),
                                  _ptr(llr), ctypes.c_uint(llr.size), _ptr(buf))
        return buf

    def pdsch_encode(self, bg, rv, qm, nof_layers, Nref, nof_ch_symbols, tb):
        tb = np.ascontiguousarray(tb, dtype=np.uint8)
        cw = np.zeros(nof_ch_symbols * qm, np.uint8)
        meta = np.zeros(4 * 200, np.uint32)
        n = self.lib.ref_pdsch_encode(bg, rv, qm, nof_layers, ctypes.c_uint(Nref), ctypes.c_uint(nof_ch_symbols),
                                      _ptr(tb), ctypes.c_uint(tb.size), _ptr(cw), _ptr(meta))
        return cw, meta[: 4 * n].reshape(n, 4)


def have_ref():
    return os.path.exists(REF_SO)


def encode_with_llrs(oracle, rng, bg, Z, crc_poly=CRC16, nof_filler=0, amp=10, noise=0.0, n_llr=None):
    """Random message with a CRC at the end of its significant bits, LDPC-encoded and mapped to LLRs."""
    K = BG_K[bg]
    L = K * Z - nof_filler
    clen = CRC_LEN[crc_poly]
    msg = np.zeros(K * Z, np.uint8)
    msg[: L - clen] = rng.integers(0, 2, L - clen)
    crc = oracle.crc_bits(crc_poly, msg[: L - clen])
    msg[L - clen: L] = [(crc >> (clen - 1 - i)) & 1 for i in range(clen)]
    cb = oracle.ldpc_encode(bg, Z, msg)
    llr = (1 - 2 * cb.astype(np.int32)) * amp
    if noise > 0:
        llr = llr + rng.normal(0, noise, llr.size)
    llr = np.clip(np.round(llr), -120, 120).astype(np.int8)
    # Filler bits are known zeros: +inf, as the rate dematcher marks them (ldpc_rate_dematcher_impl.cpp:172).
    if nof_filler:
        llr[(K - 2) * Z - nof_filler:(K - 2) * Z] = 127
    if n_llr is not None:
        llr = llr[:n_llr]
    return msg, cb, llr
