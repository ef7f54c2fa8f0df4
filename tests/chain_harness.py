"""ctypes wrapper of oracle/_ref/libsrschain.so (oracle/build_chain.sh, oracle/ref/ref_chain.cpp): the reference's own
pusch_processor_impl / pdsch_processor_impl built twice, from the reference's CPU components and with the GPU
signal-chain bindings of integration/, plus the OFDM slot transforms both ways. TEST INFRASTRUCTURE ONLY."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHAIN_SO = os.path.join(ROOT, "oracle", "_ref", "libsrschain.so")

PUSCH_CPU, PUSCH_GPU_CHAIN, PUSCH_GPU_CHAIN_HW_DEC = 0, 1, 2
PDSCH_CPU, PDSCH_GPU = 0, 1
_P = ctypes.c_void_p


class ChainParams(ctypes.Structure):
    """chain_params of oracle/ref/ref_chain.cpp."""
    _fields_ = [(n, ctypes.c_int32) for n in ("slot", "rnti", "n_id", "qm")] + [("target_code_rate", ctypes.c_float)] + \
        [(n, ctypes.c_int32) for n in ("rv", "base_graph", "new_data", "harq_id", "nof_layers", "nof_ports",
                                       "dmrs_mask", "dmrs_type2", "scrambling_id", "n_scid", "cdm_groups", "rb_start",
                                       "nof_rb", "bwp_start", "bwp_size", "start_symbol", "nof_symbols",
                                       "nof_harq_ack", "nof_csi_part1", "dc_position", "tbs_lbrm_bytes", "grid_prb",
                                       "max_iterations", "csi2_size0", "csi2_size1")]


def params(**kw):
    d = dict(slot=7, rnti=0x4601, n_id=500, qm=8, target_code_rate=948.0, rv=0, base_graph=1, new_data=1, harq_id=0,
             nof_layers=1, nof_ports=4, dmrs_mask=(1 << 2) | (1 << 11), dmrs_type2=0, scrambling_id=500, n_scid=0,
             cdm_groups=2, rb_start=0, nof_rb=25, bwp_start=0, bwp_size=273, start_symbol=0, nof_symbols=14,
             nof_harq_ack=0, nof_csi_part1=0, dc_position=-1, tbs_lbrm_bytes=200000, grid_prb=273, max_iterations=6,
             csi2_size0=0, csi2_size1=0)
    d.update(kw)
    return ChainParams(**d)


def _ptr(a):
    return a.ctypes.data_as(_P)


PUSCH_OUT = ("sch", "tb_crc_ok", "nof_cbs", "ldpc_obs", "ldpc_min", "ldpc_max", "ldpc_mean", "sinr_db", "evm", "ta_s",
             "cfo_hz", "epre_db", "rsrp_db", "uci", "harq_ack_status", "harq_ack_bits", "csi1_status", "csi1_bits")


class Chain:
    def __init__(self, device=0, max_cb_ids=128 * 160, path=CHAIN_SO):
        self.lib = ctypes.CDLL(path)
        L = self.lib
        L.chain_create.restype = _P
        L.chain_create.argtypes = [ctypes.c_int, ctypes.c_uint]
        L.chain_destroy.argtypes = [_P]
        PP = ctypes.POINTER(ChainParams)
        L.chain_ue_tx.restype = ctypes.c_int
        L.chain_ue_tx.argtypes = [_P, PP, _P, ctypes.c_uint, _P]
        L.chain_pusch_process.restype = ctypes.c_int
        L.chain_pusch_process.argtypes = [_P, ctypes.c_int, PP, _P, _P, ctypes.c_uint, _P]
        L.chain_pdsch_process.restype = ctypes.c_int
        L.chain_pdsch_process.argtypes = [_P, ctypes.c_int, PP, _P, _P, ctypes.c_uint, _P]
        L.chain_ofdm_modulate.restype = ctypes.c_int
        L.chain_ofdm_modulate.argtypes = [_P, ctypes.c_int, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint,
                                          ctypes.c_float, ctypes.c_double, ctypes.c_uint, _P, _P, ctypes.c_uint]
        L.chain_ofdm_demodulate.restype = ctypes.c_int
        L.chain_ofdm_demodulate.argtypes = [_P, ctypes.c_int, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint,
                                            ctypes.c_float, ctypes.c_double, ctypes.c_uint, ctypes.c_uint, _P,
                                            ctypes.c_uint, _P]
        self.h = L.chain_create(device, max_cb_ids)

    def close(self):
        if self.h:
            self.lib.chain_destroy(self.h)
            self.h = None

    def ue_tx(self, p, tb):
        """The UE's transmitted grid (nof_layers, 14, 12 grid_prb, 2) bf16 bit patterns."""
        tb = np.ascontiguousarray(tb, np.uint8)
        g = np.zeros((p.nof_layers, 14, 12 * p.grid_prb, 2), np.uint16)
        assert self.lib.chain_ue_tx(self.h, ctypes.byref(p), _ptr(tb), tb.size, _ptr(g)) > 0
        return g

    def pusch(self, mode, p, grid, tb_bytes):
        """pusch_processor_impl::process: (TB bytes, result dict of PUSCH_OUT)."""
        g = np.ascontiguousarray(grid, np.uint16)
        tb = np.zeros(tb_bytes, np.uint8)
        out = np.zeros(len(PUSCH_OUT), np.float64)
        assert self.lib.chain_pusch_process(self.h, mode, ctypes.byref(p), _ptr(g), _ptr(tb), tb_bytes, _ptr(out)) == 0
        return tb, dict(zip(PUSCH_OUT, out.tolist()))

    def pdsch(self, mode, p, weights, tb, grid):
        """pdsch_processor_impl::process into a copy of `grid` (nof_ports, 14, nsc, 2); returns the grid."""
        w = np.ascontiguousarray(weights, np.complex64).view(np.float32)
        tb = np.ascontiguousarray(tb, np.uint8)
        g = np.array(grid, np.uint16, copy=True, order="C")
        assert self.lib.chain_pdsch_process(self.h, mode, ctypes.byref(p), _ptr(w), _ptr(tb), tb.size, _ptr(g)) == 0
        return g

    def ofdm_modulate(self, mode, grid_port, numerology, bw_rb, dft_size, scale, center_freq_hz, slot):
        g = np.ascontiguousarray(grid_port, np.uint16)
        cap = 2 * 1024 * 1024
        out = np.zeros(cap, np.complex64)
        n = self.lib.chain_ofdm_modulate(self.h, mode, numerology, bw_rb, dft_size, scale, center_freq_hz, slot,
                                         _ptr(g), _ptr(out), cap)
        assert n > 0
        return out[:n]

    def ofdm_demodulate(self, mode, samples, numerology, bw_rb, dft_size, scale, center_freq_hz, slot,
                        window_offset=0):
        x = np.ascontiguousarray(samples, np.complex64)
        g = np.zeros((1, 14, 12 * bw_rb, 2), np.uint16)
        assert self.lib.chain_ofdm_demodulate(self.h, mode, numerology, bw_rb, dft_size, scale, center_freq_hz,
                                              window_offset, slot, _ptr(x), x.size, _ptr(g)) == 0
        return g


UL_INTS = ("rnti", "harq_id", "tb_crc_ok", "nof_cbs", "ldpc_obs", "ldpc_min", "ldpc_max", "harq_ack_status",
           "harq_ack_bits", "csi1_status", "csi1_size", "csi1_bits", "csi2_status", "csi2_size", "csi2_bits")
UL_FLOATS = ("ldpc_mean", "sinr_db", "evm", "ta_s", "cfo_hz", "epre_db", "rsrp_db")
UL_CPU, UL_GPU_BATCH = 0, 1
UL_INTERPOLATE, UL_ASYNC = 2, 4  # variant bits: estimator time strategy, asynchronous batch completion
UL_MULTI_COPY, UL_MULTI_RCCL = 8, 16  # multi-GPU batch: 3 UE shards on one device (peer copies) / RCCL world size 1
# (UL_MULTI_COPY also makes the DL batch three PDSCH shards on one device, merged into the root's grid)
DL_CPU, DL_GPU_BATCH = 0, 1


class UpperPhy:
    """The reference's own upper-PHY slot processors (uplink_processor_impl, downlink_processor_single_executor_impl)
    over the reference's CPU channel processors (variant 0) or the GPU slot batches of integration/upper_phy_gpu.cpp
    (variant 1): chain_ul_* / chain_dl_* of oracle/ref/ref_chain.cpp. TEST INFRASTRUCTURE ONLY."""

    def __init__(self, device, variant, nof_ports, grid_prb=273, max_iter=6, path=CHAIN_SO):
        self.lib = ctypes.CDLL(path)
        L = self.lib
        PP = ctypes.POINTER(ChainParams)
        L.chain_ul_create.restype = _P
        L.chain_ul_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint]
        L.chain_ul_destroy.argtypes = [_P]
        L.chain_ul_slot.restype = ctypes.c_int
        L.chain_ul_slot.argtypes = [_P, ctypes.c_uint, ctypes.c_int, PP, _P, _P, _P, _P, _P, ctypes.c_int]
        L.chain_dl_create.restype = _P
        L.chain_dl_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_uint]
        L.chain_dl_destroy.argtypes = [_P]
        L.chain_dl_slot.restype = ctypes.c_int
        L.chain_dl_slot.argtypes = [_P, ctypes.c_uint, ctypes.c_int, PP, _P, _P, _P, _P]
        L.chain_multi_transfer_counters.argtypes = [_P]
        L.chain_pdsch_transfer_counters.argtypes = [_P]
        self.P, self.grid_prb = nof_ports, grid_prb
        self.ul = L.chain_ul_create(device, variant, nof_ports, grid_prb, max_iter)
        self.dl = L.chain_dl_create(device, variant, nof_ports, grid_prb)
        assert self.ul and self.dl

    def multi_transfer_counters(self):
        """Process-wide grid transfers of the multi-device UL batches (chain_multi_transfer_counters)."""
        out = np.zeros(4, np.uint64)
        self.lib.chain_multi_transfer_counters(_ptr(out))
        return dict(zip(("host_uploads", "shard_copies", "shard_bytes", "twin_grids"), (int(v) for v in out)))

    def pdsch_transfer_counters(self):
        """Process-wide grid transfers of the PDSCH slot batches (chain_pdsch_transfer_counters)."""
        out = np.zeros(4, np.uint64)
        self.lib.chain_pdsch_transfer_counters(_ptr(out))
        return dict(zip(("grid_downloads", "shard_merges", "merge_bytes", "twin_grids"), (int(v) for v in out)))

    def close(self):
        if self.ul:
            self.lib.chain_ul_destroy(self.ul)
            self.lib.chain_dl_destroy(self.dl)
            self.ul = self.dl = None

    def ul_slot(self, slot, pdus, tb_bytes, grid):
        """One UL slot: [(result dict, payload bytes)] in notification order."""
        arr = (ChainParams * len(pdus))(*pdus)
        tbb = np.ascontiguousarray(tb_bytes, np.int32)
        g = np.ascontiguousarray(grid, np.uint16)
        n = len(pdus)
        oi = np.zeros((n, len(UL_INTS)), np.int32)
        of = np.zeros((n, 7), np.float32)
        stride = int(max(tb_bytes)) if n else 1
        tbs = np.zeros((n, stride), np.uint8)
        r = self.lib.chain_ul_slot(self.ul, slot, n, arr, _ptr(tbb), _ptr(g), _ptr(oi), _ptr(of), _ptr(tbs), stride)
        assert r >= 0, r
        out = []
        for i in range(r):
            d = dict(zip(UL_INTS, oi[i].tolist()))
            d.update(zip(UL_FLOATS, of[i].tolist()))
            out.append((d, tbs[i]))
        return out

    def dl_slot(self, slot, pdus, weights, tbs, grid):
        """One DL slot into a copy of `grid` (the other channels' content): the grid the processor sent."""
        arr = (ChainParams * len(pdus))(*pdus)
        w = np.ascontiguousarray(np.concatenate([np.asarray(x, np.complex64).ravel() for x in weights]),
                                 np.complex64).view(np.float32)
        tb = np.ascontiguousarray(np.concatenate(tbs), np.uint8)
        tbb = np.array([t.size for t in tbs], np.int32)
        g = np.array(grid, np.uint16, copy=True, order="C")
        assert self.lib.chain_dl_slot(self.dl, slot, len(pdus), arr, _ptr(w), _ptr(tb), _ptr(tbb), _ptr(g)) == 0
        return g


def factory_validate(device, direction, pdus, weights=None, path=CHAIN_SO):
    """Row b8: the GPU uplink (direction 0, PUSCH PDUs) / downlink (1, PDSCH PDUs + precoding weights) factory's
    create_pdu_validator() against the reference's own PUSCH / PDSCH validator: per PDU (factory accepts, reference
    accepts, messages differ)."""
    L = ctypes.CDLL(path)
    PP = ctypes.POINTER(ChainParams)
    L.chain_factory_validate.restype = ctypes.c_int
    L.chain_factory_validate.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, PP, _P, _P]
    arr = (ChainParams * len(pdus))(*pdus)
    w = np.zeros(2, np.float32)
    if weights:
        w = np.ascontiguousarray(np.concatenate([np.asarray(x, np.complex64).ravel() for x in weights]),
                                 np.complex64).view(np.float32)
    out = np.zeros(len(pdus), np.int32)
    assert L.chain_factory_validate(device, direction, len(pdus), arr, _ptr(w), _ptr(out)) == 0
    return [(bool(v & 1), bool(v & 2), bool(v & 4)) for v in out.tolist()]
