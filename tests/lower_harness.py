"""ctypes wrapper of the lower-PHY scenario runner in oracle/_ref/libsrschain.so (oracle/ref/ref_lower.cpp): the
reference's own pdxch_processor_impl / puxch_processor_impl on the reference's OFDM symbol transforms (variant 0) or on
the GPU symbol objects (variant 1), and the GPU PDxCH / PUxCH processors (variant 2), each driven by the same scripted
upper-PHY requests and baseband symbols. TEST INFRASTRUCTURE ONLY."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHAIN_SO = os.path.join(ROOT, "oracle", "_ref", "libsrschain.so")
_P = ctypes.c_void_p
REF_CPU, REF_ON_GPU_SYMBOLS, GPU_PROCESSOR, GPU_GROUP = 0, 1, 2, 3
# ref_lower_sectors_run variant 6: the sector group with the UL grids mapped for the device (gpu::host_blocks), as a GPU
# uplink processor's PUSCH batch maps its grid: the group demodulates into the grids' rows directly.
GPU_GROUP_MAPPED = 6
REQUEST, PROCESS = 0, 1
SENTINEL = np.float32(1e30)


def _ptr(a):
    return a.ctypes.data_as(_P)


def cp_samples(numerology, dft_size, extended, symbol_subframe):
    """cyclic_prefix::get_length (cyclic_prefix.h:93) in samples at dft_size x scs."""
    if extended:
        units = 512 >> numerology
    else:
        units = (144 >> numerology) + (16 if symbol_subframe in (0, 7 << numerology) else 0)
    return (units << numerology) * dft_size // 2048


def symbol_size(numerology, dft_size, extended, system_slot, symbol):
    nsymb = 12 if extended else 14
    return cp_samples(numerology, dft_size, extended, (system_slot % (1 << numerology)) * nsymb + symbol) + dft_size


class Lower:
    def __init__(self, path=CHAIN_SO):
        self.lib = ctypes.CDLL(path)
        f = self.lib.ref_lower_pdxch_run
        f.restype = ctypes.c_long
        f.argtypes = [ctypes.c_int] * 5 + [ctypes.c_double] + [ctypes.c_int] * 2 + [_P, _P, ctypes.c_int, _P, _P,
                                                                                      ctypes.c_long, _P, _P, _P]
        f = self.lib.ref_lower_puxch_run
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_int] * 6 + [ctypes.c_float, ctypes.c_double] + [ctypes.c_int] * 3 + [_P] * 8
        f = self.lib.ref_lower_sectors_run
        f.restype = ctypes.c_int
        f.argtypes = ([ctypes.c_int] * 7 + [ctypes.c_float, _P] + [ctypes.c_int] * 3 + [_P, _P, ctypes.c_int, _P, _P,
                      ctypes.c_long, _P, ctypes.c_int, _P, _P, ctypes.c_long] + [_P] * 8 + [ctypes.c_int, _P])

    def pdxch(self, variant, cfg, grids, port_mask, events, ring=None):
        """cfg: dict numerology, bw_rb, dft_size, extended, center_freq_hz, nof_ports. grids (G, P, nsymb, nsc, 2)
        uint16. Returns (samples complex64 in event order, processed flags, late slots). ring: benchmark mode, the
        samples go round a reused buffer of that many complex samples (returned as is, not in event order)."""
        ev = np.ascontiguousarray(np.asarray(events, np.int32).reshape(-1, 4))
        nproc = sum(e[3] - e[2] for e in ev if e[0] == PROCESS)
        cap = int(nproc * cfg["nof_ports"] * (cfg["dft_size"] * 2)) if ring is None else int(ring)
        out = np.zeros(2 * cap, np.float32)
        flags = np.zeros(max(nproc, 1), np.uint8)
        late = np.zeros(len(ev) + 1, np.int32)
        nlate = ctypes.c_int()
        g = np.ascontiguousarray(grids, np.uint16)
        m = np.ascontiguousarray(port_mask, np.uint32)
        n = self.lib.ref_lower_pdxch_run(variant, cfg["numerology"], cfg["bw_rb"], cfg["dft_size"],
                                         int(cfg["extended"]), cfg["center_freq_hz"], cfg["nof_ports"], g.shape[0],
                                         _ptr(g), _ptr(m), len(ev), _ptr(ev), _ptr(out),
                                         cap if ring is None else -cap, _ptr(flags), _ptr(late), ctypes.byref(nlate))
        assert n >= 0
        return out[: 2 * (n if ring is None else cap)].view(np.complex64), flags[:nproc], late[: nlate.value].tolist()

    def puxch(self, variant, cfg, nof_grids, events, samples, max_in_flight=2):
        """samples: complex64 of every processed symbol and port in event order. Returns (final grids
        (G, P, nsymb, nsc, 2) uint16, processed flags, [(slot, symbol)] notifications, late slots)."""
        ev = np.ascontiguousarray(np.asarray(events, np.int32).reshape(-1, 4))
        nproc = sum(e[3] - e[2] for e in ev if e[0] == PROCESS)
        nsymb = 12 if cfg["extended"] else 14
        P, nsc = cfg["nof_ports"], 12 * cfg["bw_rb"]
        grids = np.zeros((nof_grids, P, nsymb, nsc, 2), np.uint16)
        flags = np.zeros(max(nproc, 1), np.uint8)
        rx = np.zeros(2 * max(nproc, 1), np.int32)
        late = np.zeros(len(ev) + 1, np.int32)
        nrx, nlate = ctypes.c_int(), ctypes.c_int()
        x = np.ascontiguousarray(samples, np.complex64)
        r = self.lib.ref_lower_puxch_run(variant, max_in_flight, cfg["numerology"], cfg["bw_rb"], cfg["dft_size"],
                                         int(cfg["extended"]), cfg["window_offset"], cfg["center_freq_hz"], P,
                                         nof_grids, len(ev), _ptr(ev), _ptr(x), _ptr(grids), _ptr(flags), _ptr(rx),
                                         ctypes.byref(nrx), _ptr(late), ctypes.byref(nlate))
        assert r == 0
        return grids, flags[:nproc], [tuple(v) for v in rx[: 2 * nrx.value].reshape(-1, 2).tolist()], \
            late[: nlate.value].tolist()

    def sectors(self, variant, cfg, freqs, grids, masks, dl_events, ul_events, ul_samples, max_in_flight=0,
                ring=None, window_us=0, paced=False):
        """ref_lower_sectors_run: len(freqs) sectors on their own threads (variant 3: one sector group). grids
        (S, G, P, nsymb, nsc, 2) uint16 and masks (S, G): each sector's DL grids; ul_samples (S, n) complex64.
        Returns a dict: per-sector lists dl (samples, flags, late DL+UL mixed in 'late'), ul (grids, flags, rx), late,
        seconds (S, 2) DL/UL wall time, group counters (variant 3) and, paced (one symbol per symbol duration), lag
        (S, 10): DL, UL largest lag behind the pace (s), DL, UL lag at the last symbol, DL, UL fraction of symbols more
        than a slot behind, DL, UL longest process_symbol call (s), DL, UL fraction of calls longer than a symbol."""
        S = len(freqs)
        nsymb = 12 if cfg["extended"] else 14
        P = cfg["nof_ports"]
        G = grids.shape[1]
        dl_ev = np.ascontiguousarray(np.asarray(dl_events, np.int32).reshape(-1, 4))
        ul_ev = np.ascontiguousarray(np.asarray(ul_events, np.int32).reshape(-1, 4))
        n_dl = sum(e[3] - e[2] for e in dl_ev if e[0] == PROCESS)
        n_ul = sum(e[3] - e[2] for e in ul_ev if e[0] == PROCESS)
        cap = int(n_dl * P * (cfg["dft_size"] * 2)) if ring is None else int(ring)
        dl_out = np.zeros((S, 2 * cap), np.float32)
        dl_flags = np.zeros((S, max(n_dl, 1)), np.uint8)
        ul_flags = np.zeros((S, max(n_ul, 1)), np.uint8)
        ul_grids = np.zeros((S, G, P, nsymb, 12 * cfg["bw_rb"], 2), np.uint16)
        rx = np.zeros((S, 2 * max(n_ul, 1)), np.int32)
        nrx = np.zeros(S, np.int32)
        late = np.zeros((S, len(dl_ev) + len(ul_ev) + 1), np.int32)
        nlate = np.zeros(S, np.int32)
        secs = np.zeros((S, 2), np.float64)
        counts = np.zeros(8, np.uint64)
        lag = np.zeros((S, 10), np.float64)
        fr = np.ascontiguousarray(freqs, np.float64)
        g = np.ascontiguousarray(grids, np.uint16)
        m = np.ascontiguousarray(masks, np.uint32)
        x = np.ascontiguousarray(ul_samples, np.complex64)
        r = self.lib.ref_lower_sectors_run(
            variant, max_in_flight, S, cfg["numerology"], cfg["bw_rb"], cfg["dft_size"], int(cfg["extended"]),
            cfg["window_offset"], _ptr(fr), P, G, window_us, _ptr(g), _ptr(m), len(dl_ev), _ptr(dl_ev), _ptr(dl_out),
            cap if ring is None else -cap, _ptr(dl_flags), len(ul_ev), _ptr(ul_ev), _ptr(x),
            x.shape[1] if x.ndim == 2 else 0, _ptr(ul_grids), _ptr(ul_flags), _ptr(rx), _ptr(nrx), _ptr(late),
            _ptr(nlate), _ptr(secs), _ptr(counts), int(paced), _ptr(lag))
        assert r == 0
        return {
            "dl": [(dl_out[k].view(np.complex64), dl_flags[k, :n_dl]) for k in range(S)],
            "ul": [(ul_grids[k], ul_flags[k, :n_ul], [tuple(v) for v in rx[k, : 2 * nrx[k]].reshape(-1, 2).tolist()])
                   for k in range(S)],
            "late": [late[k, : nlate[k]].tolist() for k in range(S)],
            "seconds": secs,
            "lag": lag,
            "group": dict(zip(("ul_launches", "ul_batched", "ul_alone", "ul_windowed", "dl_launches", "dl_batched",
                               "dl_alone", "dl_windowed"), counts.tolist())),
        }
