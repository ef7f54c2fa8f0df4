"""Slot-level orchestration of the GPU PHY for a batch of slots of one cell: the work the reference's
upper_phy downlink processor (PDSCH processor: encoder -> DM-RS -> modulator) plus lower-PHY OFDM modulator does per
DL slot, and the uplink chain (OFDM demodulator -> DM-RS channel estimator -> PUSCH demodulator -> PUSCH decoder) per
UL slot, as plans created once and executed asynchronously on caller streams (hipGraph-capturable kernels only).

Reference call stacks (behaviour): lib/phy/upper/channel_processors/pdsch/pdsch_processor_impl.cpp (encode,
modulate, DM-RS), lib/phy/lower/modulation/ofdm_modulator_impl.cpp, lib/phy/upper/channel_processors/pusch/
pusch_processor_impl.cpp (estimate, demodulate, decode), lib/phy/lower/modulation/ofdm_demodulator_impl.cpp.

`synthesize_uplink` builds test input only (a UE transmitter + a MIMO channel + AWGN, run once before timing): it is
not part of the receive path it feeds.
"""
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

import srsgpu
from srsgpu import sch

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None

NUMEROLOGY = 1            # 30 kHz
DFT_SIZE = 4096           # 122.88 Msps
CENTER_FREQ_HZ = 3.5e9    # n78
DMRS_SYMBOL = 2           # first DM-RS symbol, type 1, two CDM groups without data
DMRS_POS1 = (1 << 2) | (1 << 11)  # dmrs-AdditionalPosition pos1: DM-RS symbols 2 and 11
DMRS_BETA = 10 ** (3 / 20)  # PUSCH / PDSCH DM-RS to data EPRE with two CDM groups without data (TS 38.214 6.2.2)
TX_SCALE = 1.0 / 64       # OFDM modulator output scaling


@dataclass
class CellSlots:
    """A batch of `nof_slots` slots of one 100 MHz 4x4 cell: the same 64 UE grants in every slot."""
    ues: List[sch.UeGrant]
    segs: List[sch.Segmentation]
    nof_slots: int
    grid_prb: int = 273
    nof_ports: int = 4
    dmrs_mask: int = 1 << DMRS_SYMBOL
    rb_first: int = 0  # first RB of the first UE (a rank's share of the UEs when a slot is sharded by UE)
    nof_symbols: int = 14  # shared-channel symbols from symbol 0 (8 in a TDD special slot's downlink part)
    slot_numbers: Optional[List[int]] = None  # slot number within the frame of each batch slot (default: s % 20)

    @property
    def nsc(self):
        return 12 * self.grid_prb

    def rb_starts(self):
        out, rb = [], self.rb_first
        for u in self.ues:
            out.append(rb)
            rb += u.n_prb
        return out

    def slot_index(self, s):
        return (s if self.slot_numbers is None else self.slot_numbers[s]) % 20

    def subframe_slots(self):
        """Slot index within the subframe of every batch slot (the OFDM phase compensation's symbol epochs)."""
        return [self.slot_index(s) % (1 << NUMEROLOGY) for s in range(self.nof_slots)]

    def grid_elems(self):
        return self.nof_slots * self.nof_ports * 14 * self.nsc


TDD_PERIOD = 10           # du_high_config.h:503-511 defaults: 10-slot period, 6 DL slots, a special slot with 8 DL
TDD_DL_SLOTS = 6          # symbols (no UL symbols) and 3 UL slots (DDDDDDSUUU)
TDD_SPECIAL_DL_SYMBOLS = 8
TDD_UL_SLOTS = 3
DMRS_POS1_8SYM = (1 << 2) | (1 << 7)  # TS 38.211 Table 7.4.1.1.2-3: type A, duration 8, pos1 -> l0 = 2 and 7


def tdd_testmode_cells(periods: int, dl_layers: int = 4, ul_layers: int = 1, mcs: int = 27, nof_prb: int = 273):
    """The du_low test mode's traffic over `periods` TDD periods of the du_high default pattern: one test UE owning the
    whole carrier in every slot (max TBS: CQI 15 -> MCS 27 of the 256QAM table, all 273 PRB), `dl_layers` PDSCH
    layers, `ul_layers` PUSCH layers, DM-RS type 1 pos1. Returns (full DL slots, special-slot DL part, UL slots) as
    CellSlots with their slot numbers in the frame (du_high_config.h:882-905 test_ue: pdsch_active / pusch_active)."""
    qm, r = sch.MCS_TABLE_256QAM[mcs]
    dl_nums = [p * TDD_PERIOD + i for p in range(periods) for i in range(TDD_DL_SLOTS)]
    sp_nums = [p * TDD_PERIOD + TDD_DL_SLOTS for p in range(periods)]
    ul_nums = [p * TDD_PERIOD + TDD_DL_SLOTS + 1 + i for p in range(periods) for i in range(TDD_UL_SLOTS)]
    dl_ue = sch.UeGrant(nof_prb, dl_layers, qm, r, nof_dmrs_symbols=2)
    sp_ue = sch.UeGrant(nof_prb, dl_layers, qm, r, nof_symb_sh=TDD_SPECIAL_DL_SYMBOLS, nof_dmrs_symbols=2)
    ul_ue = sch.UeGrant(nof_prb, ul_layers, qm, r, nof_dmrs_symbols=2)
    dl = CellSlots([dl_ue], [dl_ue.segmentation()], len(dl_nums), grid_prb=nof_prb, dmrs_mask=DMRS_POS1,
                   slot_numbers=dl_nums)
    sp = CellSlots([sp_ue], [sp_ue.segmentation()], len(sp_nums), grid_prb=nof_prb, dmrs_mask=DMRS_POS1_8SYM,
                   nof_symbols=TDD_SPECIAL_DL_SYMBOLS, slot_numbers=sp_nums)
    ul = CellSlots([ul_ue], [ul_ue.segmentation()], len(ul_nums), grid_prb=nof_prb, dmrs_mask=DMRS_POS1,
                   slot_numbers=ul_nums)
    return dl, sp, ul


def _identity(P, L):
    w = np.zeros((P, L), np.complex64)
    for i in range(min(P, L)):
        w[i, i] = 1
    return w


class DownlinkPipeline:
    """PDSCH encoder -> PDSCH DM-RS -> PDSCH modulator -> OFDM modulator for every UE of every slot."""

    def __init__(self, ctx, cell: CellSlots, weights=None, rnti0=0x4601, n_id=500, scrambling_id=500):
        self.ctx, self.cell = ctx, cell
        S, ues, segs = cell.nof_slots, cell.ues, cell.segs
        rb0 = cell.rb_starts()
        tb_bytes = [s.tbs // 8 for s in segs] * S
        enc_cfgs = [srsgpu.PdschTransportBlock(s.base_graph, 0, u.qm, u.nof_layers, u.nof_ch_symbols)
                    for u, s in zip(ues, segs)] * S
        arr, self.tb_total, self.cw_total, self.cw_offsets = srsgpu.make_pdsch_configs(tb_bytes, enc_cfgs)
        self.tb_bytes = tb_bytes
        self.encoder = srsgpu.PdschEncoderPlan(ctx, arr)
        mods, dmrs, grid_idx = [], [], []
        for s in range(S):
            for i, (u, g) in enumerate(zip(ues, segs)):
                w = _identity(cell.nof_ports, u.nof_layers) if weights is None else weights[i]
                mods.append(srsgpu.PdschModulation(
                    rnti=rnti0 + i, n_id=n_id, modulation_order=u.qm, nof_layers=u.nof_layers,
                    nof_ports=cell.nof_ports, bwp_start_rb=0, bwp_size_rb=cell.grid_prb, rb_start=rb0[i],
                    nof_rb=u.n_prb, start_symbol=0, nof_symbols=cell.nof_symbols, dmrs_symbol_mask=cell.dmrs_mask,
                    dmrs_type=1, nof_cdm_groups_without_data=2, scaling=1.0, weights=w))
                dmrs.append(srsgpu.PdschDmrs(
                    slot_index=cell.slot_index(s), scrambling_id=scrambling_id, n_scid=0, dmrs_type=1,
                    nof_layers=u.nof_layers, nof_ports=cell.nof_ports, dmrs_symbol_mask=cell.dmrs_mask,
                    reference_point_k_rb=0, rb_start=rb0[i], nof_rb=u.n_prb, amplitude=DMRS_BETA, weights=w))
                grid_idx.append(s)
        self.modulator = srsgpu.PdschModulatorPlan(ctx, srsgpu.make_pdsch_mod_configs(mods, self.cw_offsets, grid_idx),
                                                   cell.grid_prb, cell.nof_ports)
        self.dmrs = srsgpu.PdschDmrsPlan(ctx, srsgpu.make_pdsch_dmrs_configs(dmrs, grid_idx), cell.grid_prb,
                                         cell.nof_ports)
        self.ofdm = srsgpu.OfdmPlan(ctx, True, NUMEROLOGY, cell.grid_prb, DFT_SIZE, TX_SCALE, CENTER_FREQ_HZ,
                                    cell.subframe_slots(), cell.nof_ports)
        dev = torch.device("cuda", ctx.device)
        self.d_cw = torch.zeros(max(self.cw_total, 4), dtype=torch.uint8, device=dev)
        self.d_grid = torch.zeros(cell.grid_elems(), dtype=torch.int32, device=dev)
        self.d_samples = torch.zeros(2 * self.ofdm.nof_samples, dtype=torch.float32, device=dev)

    def execute(self, d_tbs, stream, events=None):
        """events: optional list of 5 torch.cuda.Event recorded between the stages on `stream`."""
        rec = (lambda i: events[i].record(stream)) if events else (lambda i: None)
        rec(0)
        self.encoder.execute(d_tbs, self.d_cw, stream)
        rec(1)
        self.dmrs.execute(self.d_grid, stream)
        self.modulator.execute(self.d_cw, self.d_grid, stream)
        rec(2)
        self.ofdm.execute(self.d_grid, self.d_samples, stream)
        rec(3)


class DownlinkGroup:
    """Several DownlinkPipelines (e.g. a TDD period's full DL slots and its special slot's DL part) run stage by stage
    on one stream, each with its own TB buffer. `fresh_tbs`: every execution first overwrites the TB payloads with
    new random bytes on the stream (graph-safe Philox: a captured graph draws new payloads on every replay), so
    consecutive slots carry fresh data like the test mode's continuous traffic."""

    def __init__(self, pipes: Sequence[DownlinkPipeline], d_tbs: Sequence, fresh_tbs=False):
        self.pipes, self.d_tbs, self.fresh_tbs = list(pipes), list(d_tbs), fresh_tbs

    def execute(self, stream, events=None, upper=True, ofdm=True, back=True):
        """upper: TB draw, encoding, DM-RS and modulation into the grids; back: the OFDM stage (modulation of the grids
        when `ofdm`). A UE-sharded cell runs the two parts as two calls, with the grid gather in between
        (srsgpu.dist.GridExchange), and only the cell's root rank modulates (ofdm=False elsewhere)."""
        rec = (lambda i: events[i].record(stream)) if events else (lambda i: None)
        if upper:
            if self.fresh_tbs:
                with torch.cuda.stream(stream):
                    for t in self.d_tbs:
                        if t.numel() % 8 == 0:  # 8 payload bytes per Philox draw (the top bit of each word stays 0)
                            t.view(torch.int64).random_()
                        else:
                            t.random_(0, 256)
            rec(0)
            for p, t in zip(self.pipes, self.d_tbs):
                p.encoder.execute(t, p.d_cw, stream)
            rec(1)
            for p in self.pipes:
                p.dmrs.execute(p.d_grid, stream)
                p.modulator.execute(p.d_cw, p.d_grid, stream)
            rec(2)
        if back:
            if ofdm:
                for p in self.pipes:
                    p.ofdm.execute(p.d_grid, p.d_samples, stream)
            rec(3)


class UplinkPipeline:
    """OFDM demodulator -> DM-RS channel estimator -> PUSCH demodulator -> PUSCH decoder for every UE of every slot.
    The channel-estimate, noise-variance, LLR, HARQ and TB buffers are owned by the pipeline. `estimate_layout`:
    srsgpu.CE_COMPACT (default: the "average" strategy's one estimate per allocation, stored once) or
    srsgpu.CE_PER_SYMBOL (the reference's channel_estimate layout); the LLRs are identical. The estimator runs du_low's
    defaults (du_low_config.h:51-69): "filter" smoothing, "average" time strategy and, with compensate_cfo, CFO
    compensation (which acts when the cell has two or more DM-RS symbols)."""

    def __init__(self, ctx, cell: CellSlots, iterations=6, rnti0=0x4601, n_id=500, scrambling_id=500,
                 equalizer=srsgpu.EQ_MMSE, estimate_layout=srsgpu.CE_COMPACT, compensate_cfo=True):
        self.ctx, self.cell, self.estimate_layout = ctx, cell, estimate_layout
        S, ues, segs = cell.nof_slots, cell.ues, cell.segs
        rb0 = cell.rb_starts()
        dev = torch.device("cuda", ctx.device)
        self.ofdm = srsgpu.OfdmPlan(ctx, False, NUMEROLOGY, cell.grid_prb, DFT_SIZE, 1.0 / (TX_SCALE * DFT_SIZE),
                                    CENTER_FREQ_HZ, cell.subframe_slots(), cell.nof_ports)
        ests, dems, grid_idx = [], [], []
        for s in range(S):
            for i, u in enumerate(ues):
                ests.append(srsgpu.PuschChannelEstimation(
                    scrambling_id=scrambling_id, n_scid=0, dmrs_type=1, nof_tx_layers=u.nof_layers,
                    nof_rx_ports=cell.nof_ports, start_symbol=0, nof_symbols=cell.nof_symbols,
                    dmrs_symbol_mask=cell.dmrs_mask, rb_start=rb0[i], nof_rb=u.n_prb, slot_index=cell.slot_index(s),
                    scaling=DMRS_BETA,
                    estimate_layout=estimate_layout, compensate_cfo=int(compensate_cfo), numerology=NUMEROLOGY))
                dems.append(srsgpu.PuschDemodulation(
                    rnti=rnti0 + i, n_id=n_id, modulation_order=u.qm, nof_tx_layers=u.nof_layers,
                    nof_rx_ports=cell.nof_ports, start_symbol=0, nof_symbols=cell.nof_symbols,
                    dmrs_symbol_mask=cell.dmrs_mask, dmrs_type=1, nof_cdm_groups_without_data=2, rb_start=rb0[i],
                    nof_rb=u.n_prb,
                    equalizer=equalizer, estimate_layout=estimate_layout, cfo_compensated=int(compensate_cfo),
                    numerology=NUMEROLOGY))
                grid_idx.append(s)
        self.chest = srsgpu.PuschChannelEstimatorPlan(ctx, srsgpu.make_pusch_chest_configs(ests, grid_idx),
                                                      cell.grid_prb, cell.nof_ports)
        darr, self.llr_offsets, self.llr_total = srsgpu.make_pusch_demod_configs(dems, grid_idx)
        self.demod = srsgpu.PuschDemodulatorPlan(ctx, darr, cell.grid_prb, cell.nof_ports)
        ul_cfgs = [srsgpu.PuschTransportBlock(s.tbs // 8, s.base_graph, 0, u.qm, u.nof_layers, u.nof_ch_symbols,
                                              nof_ldpc_iterations=iterations) for u, s in zip(ues, segs)] * S
        nof_cbs = [s.nof_segments for s in segs] * S
        cb_len = [(66 if s.base_graph == 1 else 50) * s.lifting_size for s in segs] * S
        arr, llr_total, harq_total, cb_total, tb_total = srsgpu.make_pusch_tb_configs(ul_cfgs, nof_cbs, cb_len)
        assert llr_total == self.llr_total, (llr_total, self.llr_total)
        self.decoder = srsgpu.PuschDecoderPlan(ctx, srsgpu.IMPL_SIMD, arr)
        self.tb_bytes = [s.tbs // 8 for s in segs] * S
        self.nof_tbs = len(self.tb_bytes)
        self.d_grid = torch.zeros(cell.grid_elems(), dtype=torch.int32, device=dev)
        self.d_ce = torch.zeros(4 * cell.grid_elems(), dtype=torch.int32, device=dev)
        self.d_nv = torch.zeros(4 * len(ests), dtype=torch.float32, device=dev)
        self.d_metrics = torch.zeros(4 * srsgpu.CHEST_METRICS * len(ests), dtype=torch.float32, device=dev)
        self.d_llrs = torch.zeros(max(self.llr_total, 4), dtype=torch.int8, device=dev)
        self.d_harq = torch.zeros(harq_total, dtype=torch.int8, device=dev)
        self.d_crc = torch.zeros(cb_total, dtype=torch.uint8, device=dev)
        self.d_msgs = torch.zeros(cb_total * srsgpu.CB_MSG_STRIDE, dtype=torch.uint8, device=dev)
        self.d_iters = torch.zeros(cb_total, dtype=torch.int32, device=dev)
        self.d_tbs = torch.zeros(tb_total, dtype=torch.uint8, device=dev)
        self.d_tb_ok = torch.zeros(self.nof_tbs, dtype=torch.uint8, device=dev)

    def execute(self, d_samples, stream, events=None, ofdm=True, upper=True, front=True):
        """front: the OFDM stage (demodulation of `d_samples` into the grid when `ofdm`); upper: estimation,
        demodulation and decoding of the grid. A UE-sharded cell runs the two parts as two calls with the grid scatter
        in between (srsgpu.dist.GridExchange), and only the cell's root rank demodulates (ofdm=False elsewhere)."""
        rec = (lambda i: events[i].record(stream)) if events else (lambda i: None)
        if front:
            rec(0)
            if ofdm:
                self.ofdm.execute(d_samples, self.d_grid, stream)
            rec(1)
        if not upper:
            return
        self.chest.execute(self.d_grid, self.d_ce, self.d_nv, self.d_metrics, stream)
        rec(2)
        self.demod.execute(self.d_grid, self.d_ce, self.d_nv, self.d_llrs, stream)
        rec(3)
        self.decoder.execute(self.d_llrs, self.d_harq, self.d_crc, self.d_msgs, self.d_iters, self.d_tbs,
                             self.d_tb_ok, stream)
        rec(4)


def synthesize_uplink(ctx, cell: CellSlots, d_tbs, snr_db=35.0, seed=0, rnti0=0x4601, n_id=500,
                      scrambling_id=500, cfo_hz_max=0.0):
    """Test input: the UEs' PUSCH transmissions (the same LDPC / rate matching / scrambling / modulation / layer
    mapping as the PDSCH chain, DM-RS ports 1000..1003 with amplitude beta) through a per-UE random unitary 4x4 MIMO
    channel (flat over the UE's RBs, a random phase ramp across them), a per-UE carrier frequency offset uniform in
    +-cfo_hz_max (each OFDM symbol rotated by 2 pi cfo t_l) plus AWGN at `snr_db`, OFDM-modulated into the received
    baseband samples of every slot. Returns the device sample buffer (complex float pairs)."""
    dev = torch.device("cuda", ctx.device)
    ue_tx = DownlinkPipeline(ctx, cell, weights=None, rnti0=rnti0, n_id=n_id, scrambling_id=scrambling_id)
    stream = torch.cuda.current_stream(dev)
    ue_tx.encoder.execute(d_tbs, ue_tx.d_cw, stream)
    ue_tx.dmrs.execute(ue_tx.d_grid, stream)
    ue_tx.modulator.execute(ue_tx.d_cw, ue_tx.d_grid, stream)
    torch.cuda.synchronize(dev)
    S, P, nsc = cell.nof_slots, cell.nof_ports, cell.nsc
    u = ue_tx.d_grid.view(torch.int32).reshape(S, P, 14, nsc)
    x = torch.complex(((u << 16).view(torch.float32)), ((u & -65536).view(torch.float32)))  # bf16 pairs -> complex
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    # Per-subcarrier 4x4 channel: each UE's random unitary matrix (QR of a complex Gaussian) and a phase ramp.
    H = torch.zeros(nsc, P, P, dtype=torch.complex64, device=dev)
    k0 = 0
    for ue in cell.ues:
        g = torch.complex(torch.randn(P, P, generator=gen, device=dev), torch.randn(P, P, generator=gen, device=dev))
        q, _ = torch.linalg.qr(g)
        k1 = k0 + 12 * ue.n_prb
        ramp = torch.exp(1j * 2 * torch.pi * torch.arange(k1 - k0, device=dev) * float(torch.rand(1, generator=gen,
                                                                                                device=dev)) / 256)
        H[k0:k1] = q[None] * ramp[:, None, None]
        k0 = k1
    y = torch.einsum("kpl,slmk->spmk", H, x)
    if cfo_hz_max > 0:
        t = torch.zeros(14, dtype=torch.float64)
        scs_hz = (15 << NUMEROLOGY) * 1000.0
        for i in range(14):  # symbol start epochs in symbol durations (normal CP)
            kappa = (144 >> NUMEROLOGY) + (16 if i in (0, 7 << NUMEROLOGY) else 0)
            d = kappa * 64 / (480000 * 4096) * scs_hz
            t[i] = d if i == 0 else t[i - 1] + d + 1.0
        cfo = torch.zeros(nsc, dtype=torch.float64)
        k0 = 0
        for ue in cell.ues:
            k1 = k0 + 12 * ue.n_prb
            cfo[k0:k1] = (float(torch.rand(1, generator=gen, device=dev)) * 2 - 1) * cfo_hz_max / scs_hz
            k0 = k1
        rot = torch.exp(2j * torch.pi * t[:, None] * cfo[None, :]).to(torch.complex64).to(dev)  # (14, nsc)
        y = y * rot[None, None]
    nv = 10 ** (-snr_db / 10)
    y = y + torch.complex(torch.randn(y.shape, generator=gen, device=dev),
                          torch.randn(y.shape, generator=gen, device=dev)) * float(np.sqrt(nv / 2))
    yr = y.real.float().contiguous()
    yi = y.imag.float().contiguous()

    def to_bf16(v):  # round half to even on the bit pattern
        b = v.view(torch.int32)
        return (b + 0x7FFF + ((b >> 16) & 1)) >> 16

    rx_grid = ((to_bf16(yr) & 0xFFFF) | (to_bf16(yi) << 16)).to(torch.int32).contiguous().reshape(-1)
    air = srsgpu.OfdmPlan(ctx, True, NUMEROLOGY, cell.grid_prb, DFT_SIZE, TX_SCALE, CENTER_FREQ_HZ,
                          cell.subframe_slots(), P)
    d_samples = torch.zeros(2 * air.nof_samples, dtype=torch.float32, device=dev)
    air.execute(rx_grid, d_samples, stream)
    torch.cuda.synchronize(dev)
    air.close()
    return d_samples
