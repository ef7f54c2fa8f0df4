"""ctypes wrapper of oracle/_ref/libsrshal.so (oracle/build_hal.sh, oracle/ref/ref_hal.cpp): the reference's own
pusch_decoder_impl / pusch_decoder_hw_impl / pdsch_encoder_impl / pdsch_encoder_hw_impl with the GPU bindings of
integration/ plugged in. TEST INFRASTRUCTURE ONLY."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HAL_SO = os.path.join(ROOT, "oracle", "_ref", "libsrshal.so")

PUSCH_CPU, PUSCH_SW_GPU_LDPC, PUSCH_HW_GPU = 0, 1, 2   # hal_pusch_decode modes
PDSCH_CPU, PDSCH_HW_GPU = 0, 1                          # hal_pdsch_encode modes
_P = ctypes.c_void_p


def _ptr(a):
    return a.ctypes.data_as(_P)


class Hal:
    def __init__(self, device=0, max_cb_ids=64 * 160, path=HAL_SO):
        self.lib = ctypes.CDLL(path)
        self.lib.hal_create.restype = _P
        self.lib.hal_create.argtypes = [ctypes.c_int, ctypes.c_uint]
        self.lib.hal_destroy.argtypes = [_P]
        self.lib.hal_pusch_decode.restype = ctypes.c_int
        self.lib.hal_pusch_decode.argtypes = [_P, ctypes.c_int, ctypes.c_uint, ctypes.c_uint] + [ctypes.c_int] * 4 + \
            [ctypes.c_uint] + [ctypes.c_int] * 3 + [_P, ctypes.c_uint, _P, ctypes.c_uint, _P]
        self.lib.hal_pdsch_encode.restype = ctypes.c_int
        self.lib.hal_pdsch_encode.argtypes = [_P] + [ctypes.c_int] * 5 + [ctypes.c_uint, ctypes.c_uint, _P,
                                                                            ctypes.c_uint, _P]
        self.h = self.lib.hal_create(device, max_cb_ids)

    def close(self):
        if self.h:
            self.lib.hal_destroy(self.h)
            self.h = None

    def pusch_decode(self, mode, harq_id, nof_cbs, bg, rv, qm, nof_layers, llrs, tb_bytes, new_data=True, Nref=0,
                     max_iter=6, early_stop=True):
        """Returns (tb bytes, stats dict: tb_crc_ok, nof_cbs, nof_obs, min, max, mean iterations)."""
        llrs = np.ascontiguousarray(llrs, np.int8)
        tb = np.zeros(tb_bytes, np.uint8)
        st = np.zeros(6, np.float64)
        r = self.lib.hal_pusch_decode(self.h, mode, harq_id, nof_cbs, bg, rv, qm, nof_layers, Nref, max_iter,
                                      int(early_stop), int(new_data), _ptr(llrs), llrs.size, _ptr(tb), tb_bytes,
                                      _ptr(st))
        assert r == 0, "the decoder did not notify"
        return tb, dict(tb_crc_ok=bool(st[0]), nof_cbs=int(st[1]), nof_obs=int(st[2]), min=st[3], max=st[4],
                        mean=st[5])

    def pdsch_encode(self, mode, bg, rv, qm, nof_layers, nof_ch_symbols, tb, Nref=0):
        """Returns the codeword, one bit per byte."""
        tb = np.ascontiguousarray(tb, np.uint8)
        cw = np.zeros(nof_ch_symbols * qm, np.uint8)
        assert self.lib.hal_pdsch_encode(self.h, mode, bg, rv, qm, nof_layers, nof_ch_symbols, Nref, _ptr(tb),
                                         tb.size, _ptr(cw)) == 0
        return cw


class HalPool:
    """hal_pool_*: `nof_threads` persistent worker threads, each with its own reference pusch_decoder_hw_impl over ONE
    shared hw_decoder_pool of GPU accelerators (made by a factory destroyed before any decode), plus the reference CPU
    decoder. decode(worker=-1) runs the CPU reference; worker >= 0 runs on that thread (its own pool accelerator)."""

    def __init__(self, device=0, max_cb_ids=64 * 160, nof_threads=4, path=HAL_SO):
        self.lib = ctypes.CDLL(path)
        self.lib.hal_pool_create.restype = _P
        self.lib.hal_pool_create.argtypes = [ctypes.c_int, ctypes.c_uint, ctypes.c_uint]
        self.lib.hal_pool_destroy.argtypes = [_P]
        self.lib.hal_pool_decode.restype = ctypes.c_int
        self.lib.hal_pool_decode.argtypes = [_P, ctypes.c_int, ctypes.c_uint, ctypes.c_uint] + [ctypes.c_int] * 4 + \
            [ctypes.c_uint] + [ctypes.c_int] * 3 + [_P, ctypes.c_uint, _P, ctypes.c_uint, _P]
        self.h = self.lib.hal_pool_create(device, max_cb_ids, nof_threads)

    def close(self):
        if self.h:
            self.lib.hal_pool_destroy(self.h)
            self.h = None

    def decode(self, worker, harq_id, nof_cbs, bg, rv, qm, nof_layers, llrs, tb_bytes, new_data=True, Nref=0,
               max_iter=6, early_stop=True):
        llrs = np.ascontiguousarray(llrs, np.int8)
        tb = np.zeros(tb_bytes, np.uint8)
        st = np.zeros(6, np.float64)
        r = self.lib.hal_pool_decode(self.h, worker, harq_id, nof_cbs, bg, rv, qm, nof_layers, Nref, max_iter,
                                     int(early_stop), int(new_data), _ptr(llrs), llrs.size, _ptr(tb), tb_bytes,
                                     _ptr(st))
        assert r == 0, f"the decoder did not notify ({r})"
        return tb, dict(tb_crc_ok=bool(st[0]), nof_cbs=int(st[1]), nof_obs=int(st[2]), min=st[3], max=st[4],
                        mean=st[5])
