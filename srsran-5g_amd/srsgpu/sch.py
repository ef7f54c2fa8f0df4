"""Shared-channel (SCH) host logic: transport-block size and LDPC segmentation.

Host-side mirrors (no compute kernels) of
  * TS 38.214 §5.1.3.2 TBS determination       — reference lib/ran/sch/tbs_calculator.cpp:26-:110
  * LDPC base-graph selection, TS 38.212 §7.2.2 — reference include/srsran/ran/sch/ldpc_base_graph.h:38
  * LDPC segmentation, TS 38.212 §5.2.2/§5.4.2 — reference lib/phy/upper/channel_coding/ldpc/
    ldpc_segmenter_tx_impl.cpp:58 (new_transmission) and ldpc_segmenter_helpers.h:75 (rm lengths)
used to describe the codeblocks a PDSCH/PUSCH transport block is split into. tests/test_sch.py pins the segmentation
against the reference build.
"""
import math
from dataclasses import dataclass, field
from typing import List

LIFTING_SIZES = [2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 20, 22, 24, 26, 28, 30, 32, 36, 40, 44, 48,
                 52, 56, 60, 64, 72, 80, 88, 96, 104, 112, 120, 128, 144, 160, 176, 192, 208, 224, 240, 256, 288, 320,
                 352, 384]

# TS 38.214 Table 5.1.3.2-1: TBS for N_info <= 3824.
_TBS_TABLE = [24, 32, 40, 48, 56, 64, 72, 80, 88, 96, 104, 112, 120, 128, 136, 144, 152, 160, 168, 176, 184, 192, 208,
              224, 240, 256, 272, 288, 304, 320, 336, 352, 368, 384, 408, 432, 456, 480, 504, 528, 552, 576, 608, 640,
              672, 704, 736, 768, 808, 848, 888, 928, 984, 1032, 1064, 1128, 1160, 1192, 1224, 1256, 1288, 1320, 1352,
              1416, 1480, 1544, 1608, 1672, 1736, 1800, 1864, 1928, 2024, 2088, 2152, 2216, 2280, 2408, 2472, 2536,
              2600, 2664, 2728, 2792, 2856, 2976, 3104, 3240, 3368, 3496, 3624, 3752, 3824]

# TS 38.214 Table 5.1.3.1-2 (MCS index table 2, 256QAM): index -> (Qm, R x 1024).
MCS_TABLE_256QAM = {
    0: (2, 120), 1: (2, 193), 2: (2, 308), 3: (2, 449), 4: (2, 602), 5: (4, 378), 6: (4, 434), 7: (4, 490),
    8: (4, 553), 9: (4, 616), 10: (4, 658), 11: (6, 466), 12: (6, 517), 13: (6, 567), 14: (6, 616), 15: (6, 666),
    16: (6, 719), 17: (6, 772), 18: (6, 822), 19: (6, 873), 20: (8, 682.5), 21: (8, 711), 22: (8, 754), 23: (8, 797),
    24: (8, 841), 25: (8, 885), 26: (8, 916.5), 27: (8, 948),
}
# TS 38.214 Table 5.1.3.1-1 (MCS index table 1, 64QAM).
MCS_TABLE_64QAM = {
    0: (2, 120), 1: (2, 157), 2: (2, 193), 3: (2, 251), 4: (2, 308), 5: (2, 379), 6: (2, 449), 7: (2, 526),
    8: (2, 602), 9: (2, 679), 10: (4, 340), 11: (4, 378), 12: (4, 434), 13: (4, 490), 14: (4, 553), 15: (4, 616),
    16: (4, 658), 17: (6, 438), 18: (6, 466), 19: (6, 517), 20: (6, 567), 21: (6, 616), 22: (6, 666), 23: (6, 719),
    24: (6, 772), 25: (6, 822), 26: (6, 873), 27: (6, 910), 28: (6, 948),
}


def _f32(x):
    """Rounds to IEEE single precision (the reference computes the TBS in float)."""
    import struct
    return struct.unpack("f", struct.pack("f", x))[0]


def tbs_calculate(n_prb: int, nof_symb_sh: int, nof_dmrs_prb: int, nof_oh_prb: int, qm: int, r1024: float,
                  nof_layers: int, tb_scaling: int = 0) -> int:
    """TS 38.214 §5.1.3.2 (tbs_calculator.cpp:100 tbs_calculator_calculate)."""
    nof_re_prime = 12 * nof_symb_sh - nof_dmrs_prb - nof_oh_prb
    nof_re = min(nof_re_prime, 156) * n_prb
    scaling = 1.0 / (1 << tb_scaling)
    tcr = _f32(r1024 / 1024.0)
    nof_info = _f32(_f32(_f32(_f32(scaling * nof_re) * tcr) * qm) * nof_layers)
    if nof_info <= 3824:
        n = 3 if nof_info <= 512 else int(math.floor(math.log2(nof_info))) - 6
        info_p = max(24, (1 << n) * int(math.floor(nof_info / (1 << n))))
        for t in _TBS_TABLE:
            if t >= info_p:
                return t
        raise ValueError("TBS table overflow")
    n = int(math.floor(math.log2(nof_info - 24)) - 5)
    info_p = max(3840, (1 << n) * int(round((nof_info - 24) / (1 << n))))
    if tcr <= 0.25:
        C = -(-(info_p + 24) // 3816)
    elif info_p > 8424:
        C = -(-(info_p + 24) // 8424)
    else:
        C = 1
    return 8 * C * (-(-(info_p + 24) // (8 * C))) - 24


def base_graph(tbs: int, r: float) -> int:
    """ldpc_base_graph.h:38 get_ldpc_base_graph."""
    if tbs <= 292 or r <= 0.25 or (tbs <= 3824 and r <= 0.67):
        return 2
    return 1


def tb_crc_size(tbs: int) -> int:
    return 16 if tbs <= 3824 else 24


@dataclass
class Codeblock:
    index: int
    lifting_size: int
    nof_filler_bits: int
    rm_length: int            # E
    cw_offset: int            # first bit of this codeblock in the codeword
    tb_offset: int            # first TB(+CRC) bit carried by this codeblock
    nof_info_bits: int        # TB(+TB CRC) bits carried (cb_info_bits, without CB CRC)
    nof_crc_bits: int         # codeblock CRC length carried in the decoder config (16/24)


@dataclass
class Segmentation:
    tbs: int
    base_graph: int
    nof_segments: int
    lifting_size: int
    segment_length: int       # K (= 22 Z or 10 Z)
    nof_filler_bits: int
    nof_tb_crc_bits: int
    cb_crc_bits: int          # 24 when segmented, else 0
    zero_pad: int
    cw_length: int
    codeblocks: List[Codeblock] = field(default_factory=list)


def segment(tbs: int, bg: int, qm: int, nof_layers: int, nof_ch_symbols: int) -> Segmentation:
    """ldpc_segmenter_tx_impl.cpp:58 new_transmission (TS 38.212 §5.2.2 code block segmentation + §5.4.2.1 E)."""
    assert tbs % 8 == 0 and nof_ch_symbols % nof_layers == 0
    tb_crc = tb_crc_size(tbs)
    b_in = tbs + tb_crc
    max_seg = 8448 if bg == 1 else 3840
    C = 1 if b_in <= max_seg else -(-b_in // (max_seg - 24))
    b_out = b_in + (24 * C if C > 1 else 0)
    # compute_lifting_size (ldpc.h:166)
    if bg == 1:
        kb = 22
    elif b_in > 640:
        kb = 10
    elif b_in > 560:
        kb = 9
    elif b_in > 192:
        kb = 8
    else:
        kb = 6
    Z = next(z for z in LIFTING_SIZES if z * kb * C >= b_out)
    K = (22 if bg == 1 else 10) * Z
    cb_crc = 24 if C > 1 else 0
    cb_info = -(-b_out // C) - cb_crc
    zero_pad = (cb_info + cb_crc) * C - b_out
    sym_per_layer = nof_ch_symbols // nof_layers
    nof_short = C - (sym_per_layer % C)
    filler = K - cb_info - cb_crc
    seg = Segmentation(tbs, bg, C, Z, K, filler, tb_crc, cb_crc, zero_pad, nof_ch_symbols * qm)
    cw_off = 0
    tb_off = 0
    for i in range(C):
        if i < nof_short:
            E = (sym_per_layer // C) * nof_layers * qm
        else:
            E = (-(-sym_per_layer // C)) * nof_layers * qm
        used = cb_info - ((tb_crc + zero_pad) if i == C - 1 else 0)
        seg.codeblocks.append(Codeblock(i, Z, filler, E, cw_off, tb_off, used, tb_crc if C == 1 else cb_crc))
        tb_off += used + (tb_crc if i == C - 1 else 0)
        cw_off += E
    assert cw_off == seg.cw_length and tb_off == b_in
    return seg


@dataclass
class UeGrant:
    """One UE's PUSCH/PDSCH allocation in a slot."""
    n_prb: int
    nof_layers: int
    qm: int
    r1024: float
    nof_symb_sh: int = 14
    nof_dmrs_symbols: int = 1

    @property
    def nof_ch_symbols(self) -> int:
        # Data REs: DM-RS symbols carry no data (two CDM groups without data, type 1).
        return self.n_prb * 12 * (self.nof_symb_sh - self.nof_dmrs_symbols) * self.nof_layers

    @property
    def tbs(self) -> int:
        return tbs_calculate(self.n_prb, self.nof_symb_sh, 12 * self.nof_dmrs_symbols, 0, self.qm, self.r1024,
                             self.nof_layers)

    def segmentation(self) -> Segmentation:
        tbs = self.tbs
        return segment(tbs, base_graph(tbs, self.r1024 / 1024.0), self.qm, self.nof_layers, self.nof_ch_symbols)


def slot_100mhz_4x4(nof_ues: int = 64, mcs: int = 27, nof_prb: int = 273, nof_layers: int = 4,
                    nof_dmrs_symbols: int = 1) -> List[UeGrant]:
    """n78 100 MHz (30 kHz SCS, 273 PRB) slot shared by `nof_ues` UEs, `nof_layers` layers, MCS table 2 (256QAM),
    `nof_dmrs_symbols` DM-RS symbols (type 1, two CDM groups without data)."""
    qm, r = MCS_TABLE_256QAM[mcs]
    base = nof_prb // nof_ues
    extra = nof_prb - base * nof_ues
    return [UeGrant(base + (1 if i < extra else 0), nof_layers, qm, r, nof_dmrs_symbols=nof_dmrs_symbols)
            for i in range(nof_ues)]
