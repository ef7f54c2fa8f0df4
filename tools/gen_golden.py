#!/usr/bin/env python3
"""Generates tests/golden/*.npz: input/output vectors produced by the srsRAN reference itself (built from its own
sources by oracle/build_ref.sh into oracle/_ref/libsrsref.so). The reference repository ships no test-vector archives
(its CMake downloads *_test_data.tar.gz at build time), so these fixtures are the pinned reference outputs; they travel
to the GPU box where /root/reference does not exist.

Run: python tools/gen_golden.py   (deterministic: fixed seeds)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "srsran-5g_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from oracle_lib import BG_K, BG_N_SHORT, CRC16, CRC24A, CRC24B, CRC_LEN, Reference  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def ref_encode_llrs(ref, rng, bg, Z, crc_poly, nof_filler, amp, noise, n_llr):
    """Message with CRC (computed by the reference CRC), encoded by the reference encoder, mapped to LLRs."""
    K = BG_K[bg]
    L = K * Z - nof_filler
    clen = CRC_LEN[crc_poly]
    msg = np.zeros(K * Z, np.uint8)
    msg[: L - clen] = rng.integers(0, 2, L - clen)
    crc = ref.crc_bits(crc_poly, msg[: L - clen])
    msg[L - clen: L] = [(crc >> (clen - 1 - i)) & 1 for i in range(clen)]
    cb = ref.ldpc_encode(bg, Z, msg)
    llr = (1 - 2 * cb.astype(np.int32)) * amp + (rng.normal(0, noise, cb.size) if noise > 0 else 0)
    llr = np.clip(np.round(llr), -120, 120).astype(np.int8)
    if nof_filler:
        llr[(K - 2) * Z - nof_filler:(K - 2) * Z] = 127
    return llr[:n_llr]


def gen_crc(ref, rng):
    polys, bits_list, want = [], [], []
    for poly in range(6):
        for n in (1, 24, 100, 1000, 8448):
            b = rng.integers(0, 2, n).astype(np.uint8)
            polys.append(poly)
            bits_list.append(b)
            want.append(ref.crc_bits(poly, b))
    lens = np.array([b.size for b in bits_list], np.int32)
    np.savez_compressed(os.path.join(OUT, "crc.npz"), poly=np.array(polys, np.int32), lens=lens,
                        bits=np.concatenate(bits_list), crc=np.array(want, np.uint32))


def gen_encoder(ref, rng):
    rows = []
    msgs, cbs = [], []
    for bg in (1, 2):
        for Z in (2, 7, 15, 36, 104, 208, 224, 240, 288, 320, 352, 384):
            msg = rng.integers(0, 2, BG_K[bg] * Z).astype(np.uint8)
            cb = ref.ldpc_encode(bg, Z, msg)
            rows.append((bg, Z))
            msgs.append(np.packbits(msg))
            cbs.append(np.packbits(cb))
    np.savez_compressed(os.path.join(OUT, "ldpc_encoder.npz"), cfg=np.array(rows, np.int32),
                        msg=np.concatenate(msgs), cb=np.concatenate(cbs))


def gen_decoder(ref, rng):
    """Cases: (bg, Z, impl, crc_poly or -1, nof_crc_bits, filler, max_iter, scaling) + LLRs -> (iters, bits)."""
    cfg, llrs, iters, outs = [], [], [], []
    cases = []
    for bg in (1, 2):
        for Z in (2, 5, 13, 24, 64, 112, 208, 288, 352, 384):
            for trial in range(4):
                cases.append((bg, Z, trial))
    for bg, Z, trial in cases:
        K, N = BG_K[bg], BG_N_SHORT[bg]
        crc_poly = [CRC16, CRC24B, CRC24A, CRC24B][trial]
        filler = 0 if trial in (0, 1) else min(Z, (K - 2) * Z // 6)
        if K * Z - filler < CRC_LEN[crc_poly] + 8:
            crc_poly = 5
        noise = [0.0, 7.0, 10.0, 14.0][trial]
        n_nodes = [N, K + 2, (K + N) // 2, N][trial]
        llr = ref_encode_llrs(ref, rng, bg, Z, crc_poly, filler, 12, noise, n_nodes * Z)
        for impl in (Reference.GENERIC, Reference.AVX2):
            for use_crc in (True, False):
                if not use_crc and trial % 2:
                    continue
                nbits = 16 if CRC_LEN[crc_poly] < 24 else 24
                r, o = ref.ldpc_decode(impl, bg, Z, llr, nof_crc_bits=nbits, nof_filler=filler,
                                       crc_poly=crc_poly if use_crc else -1, max_iter=8, scaling=0.8)
                cfg.append((bg, Z, impl, crc_poly if use_crc else -1, nbits, filler, 8, len(llr)))
                llrs.append(llr)
                iters.append(r)
                outs.append(np.packbits(o))
    np.savez_compressed(os.path.join(OUT, "ldpc_decoder.npz"), cfg=np.array(cfg, np.int32),
                        llr=np.concatenate(llrs), iters=np.array(iters, np.int32), out=np.concatenate(outs))


def gen_rate_matching(ref, rng):
    """Per case: message, rate-matched output, dematcher input/initial buffer and the four dematcher outputs
    (new_data 1/0 x generic/SIMD combining)."""
    cfg, msgs, rm_out, dm_llr, dm_init, dm_out = [], [], [], [], [], []
    for bg in (1, 2):
        for Z in (3, 16, 64, 208, 384):
            for rv in range(4):
                if Z == 384 and rv in (1, 2):
                    continue
                qm = [1, 2, 4, 6, 8][(Z + rv) % 5]
                N = BG_N_SHORT[bg] * Z
                nsys = (BG_K[bg] - 2) * Z
                filler = int(rng.integers(0, max(1, nsys // 4)))
                Nref = [0, int(N * 0.75)][(rv + bg) % 2]
                E = qm * int(rng.integers(max(1, (BG_K[bg] * Z) // qm // 2), 2 * N // qm))
                msg = rng.integers(0, 2, BG_K[bg] * Z).astype(np.uint8)
                msg[BG_K[bg] * Z - filler:] = 0
                out = ref.rate_match(bg, Z, rv, qm, Nref, filler, msg, E)
                llr = rng.integers(-120, 121, E).astype(np.int8)
                init = rng.integers(-120, 121, N).astype(np.int8)
                cfg.append((bg, Z, rv, qm, Nref, filler, E))
                msgs.append(np.packbits(msg))
                rm_out.append(np.packbits(out))
                dm_llr.append(llr)
                dm_init.append(init)
                for new_data in (1, 0):
                    for impl in (0, 1):
                        dm_out.append(ref.rate_dematch(impl, bg, Z, rv, qm, Nref, filler, new_data, llr, init))
    np.savez_compressed(os.path.join(OUT, "rate_matching.npz"), cfg=np.array(cfg, np.int32),
                        msg=np.concatenate(msgs), rm_out=np.concatenate(rm_out), dm_llr=np.concatenate(dm_llr),
                        dm_init=np.concatenate(dm_init), dm_out=np.concatenate(dm_out))


def gen_pdsch_encoder(ref, rng):
    from srsgpu import sch
    cfg, tbs, cws, metas = [], [], [], []
    for (n_prb, layers, qm, r) in ((4, 4, 8, 948), (5, 4, 8, 948), (51, 1, 6, 772), (10, 2, 4, 434), (2, 1, 2, 120),
                                   (24, 3, 6, 517), (106, 2, 8, 682.5)):
        g = sch.UeGrant(n_prb, layers, qm, r)
        seg = g.segmentation()
        for rv in (0, 2):
            tb = rng.integers(0, 256, seg.tbs // 8).astype(np.uint8)
            cw, meta = ref.pdsch_encode(seg.base_graph, rv, qm, layers, 0, g.nof_ch_symbols, tb)
            cfg.append((seg.base_graph, rv, qm, layers, 0, g.nof_ch_symbols, seg.tbs // 8, meta.shape[0]))
            tbs.append(tb)
            cws.append(np.packbits(cw))
            metas.append(meta.astype(np.int32))
    np.savez_compressed(os.path.join(OUT, "pdsch_encoder.npz"), cfg=np.array(cfg, np.int32), tb=np.concatenate(tbs),
                        cw=np.concatenate(cws), meta=np.concatenate(metas))


def gen_pdsch_modulator(ref, rng):
    from oracle_lib import PDSCH_MOD_KEYS
    from pdsch_mod_cases import random_config
    grid_prb = 24
    cfgs, scal, ws, cws, grids = [], [], [], [], []
    for i in range(12):
        cfg, nbits, w = random_config(rng, grid_prb, qm=[2, 4, 6, 8][i % 4])
        cw = rng.integers(0, 256, (nbits + 7) // 8).astype(np.uint8)
        grid = ref.pdsch_modulate(cfg, w, cw, nbits, grid_prb)
        cfgs.append([cfg[k] for k in PDSCH_MOD_KEYS[:-1]] + [nbits, grid_prb])
        scal.append(cfg["scaling"])
        ws.append(w.ravel())
        cws.append(cw)
        grids.append(grid.ravel())
    np.savez_compressed(os.path.join(OUT, "pdsch_modulator.npz"), cfg=np.array(cfgs, np.int64),
                        scaling=np.array(scal, np.float32), weights=np.concatenate(ws), cw=np.concatenate(cws),
                        grid=np.concatenate(grids))


GOLDEN_OFDM_CASES = [(3, 2), (5, 1), (8, 2), (0, 1), (6, 1)]  # (index into ofdm_cases.CASES, ports)


def gen_ofdm(ref, rng):
    """Reference OFDM slot modulator output of random bf16 grids, and the reference demodulator's grid of those
    samples (scale 1 / (scale * N): the round trip returns the input grid up to bf16 rounding)."""
    from ofdm_cases import CASES, random_grid
    out = {}
    for i, (c, P) in enumerate(GOLDEN_OFDM_CASES):
        mu, rb, N, ext, scale, fc, slot, woff = CASES[c]
        ns = 12 if ext else 14
        grid = random_grid(rng, P, ns, 12 * rb, occupancy=0.9)
        x = ref.ofdm_modulate(grid, mu, rb, N, ext, scale, fc, slot)
        g2 = ref.ofdm_demodulate(x, mu, rb, N, ext, 1.0 / (scale * N), fc, slot, woff)
        out[f"case{i}_grid"] = grid
        out[f"case{i}_samples"] = x
        out[f"case{i}_demod"] = g2
        out[f"case{i}_params"] = np.array([c, P], np.int64)
    np.savez_compressed(os.path.join(OUT, "ofdm.npz"), **out)


def gen_pusch_demod(ref, rng):
    """Reference PUSCH demodulator LLRs (pusch_demodulator_impl, generic equalizer ZF / MMSE, SIMD demapper) of random
    transmissions in 24-PRB grids, and reference demapper LLRs of random symbols for every modulation."""
    from pusch_demod_cases import random_case
    out = {}
    specs = [(1, 1, 2), (1, 2, 4), (1, 4, 6), (1, 3, 8), (2, 2, 8), (2, 4, 6), (2, 2, 4), (2, 4, 2), (1, 4, 8)]
    for i, (L, P, qm) in enumerate(specs):
        cfg, grid, H, nv = random_case(rng, 24, nof_layers=L, nof_rx_ports=P, qm=qm)
        mmse = i == 8
        llr = ref.pusch_demodulate(cfg, grid, H, nv, 24, mmse)
        out[f"case{i}_cfg"] = np.array([cfg[k] for k in PUSCH_DEMOD_KEYS] + [int(mmse)], np.int64)
        out[f"case{i}_grid"], out[f"case{i}_ch_est"], out[f"case{i}_noise_var"] = grid, H, nv
        out[f"case{i}_llr"] = llr
    for qm in (2, 4, 6, 8):
        n = 4000
        x = (rng.uniform(-1.5, 1.5, n) + 1j * rng.uniform(-1.5, 1.5, n)).astype(np.complex64)
        x[::97] = 0
        nvar = rng.uniform(0.001, 0.5, n).astype(np.float32)
        nvar[::89] = 0
        out[f"demap{qm}_symbols"], out[f"demap{qm}_noise_var"] = x, nvar
        out[f"demap{qm}_llr"] = ref.demodulate_soft(qm, x, nvar)
    np.savez_compressed(os.path.join(OUT, "pusch_demod.npz"), **out)


def gen_pusch_demod_general(ref, rng):
    """Reference PUSCH demodulator LLRs and statistics (per-symbol / end post-equalization SINR and EVM) with general
    CRB masks and transform precoding, in 32-PRB grids."""
    from pusch_demod_cases import random_general_case
    out = {}
    specs = [(False, True, None), (True, True, None), (True, False, None), (False, True, 1), (True, True, 5),
             (False, False, 32), (True, False, 32), (False, True, 16)]
    for i, (tp, mask, max_rb) in enumerate(specs):
        cfg, grid, H, nv, crb = random_general_case(rng, 32, transform_precoding=tp, mask=mask, max_rb=max_rb)
        llr, stats = ref.pusch_demodulate_ex(cfg, grid, H, nv, 32, crb_mask=crb, transform_precoding=tp)
        out[f"case{i}_cfg"] = np.array([cfg[k] for k in PUSCH_DEMOD_KEYS] + [int(tp)], np.int64)
        out[f"case{i}_crb"] = crb if crb is not None else np.zeros(0, np.uint8)
        out[f"case{i}_grid"], out[f"case{i}_ch_est"], out[f"case{i}_noise_var"] = grid, H, nv
        out[f"case{i}_llr"], out[f"case{i}_stats"] = llr, stats
    np.savez_compressed(os.path.join(OUT, "pusch_demod_general.npz"), **out)


def gen_ulsch_demux(ref, rng):
    """Reference UL-SCH demultiplexer outputs (ulsch_demultiplex_impl) of random UCI-on-PUSCH configurations."""
    from ulsch_demux_cases import nof_llrs, random_config
    out = {}
    for i in range(12):
        cfg, c2b, c2e, c_init = random_config(rng)
        llrs = rng.integers(-120, 121, nof_llrs(cfg)).astype(np.int8)
        res = ref.ulsch_demux(cfg, llrs, c_init, c2b, c2e, block_size=int(rng.integers(7, 500)))
        out[f"case{i}_cfg"] = np.array([cfg[k] for k in ULSCH_DEMUX_KEYS] + [c2b, c2e, c_init], np.int64)
        out[f"case{i}_llrs"] = llrs
        for k, v in res.items():
            out[f"case{i}_{k}"] = v
    np.savez_compressed(os.path.join(OUT, "ulsch_demux.npz"), **out)


ULSCH_DEMUX_KEYS = ["qm", "nof_layers", "nof_prb", "start_symbol", "nof_symbols", "dmrs_symbol_mask", "dmrs_type2",
                    "nof_cdm_groups_without_data", "nof_harq_ack_rvd", "nof_harq_ack_bits", "nof_enc_harq_ack_bits",
                    "nof_csi_part1_bits", "nof_enc_csi_part1_bits"]


def gen_pusch_chest(ref, rng):
    """Reference DM-RS channel estimates (dmrs_pusch_estimator_impl, filter / mean / none smoothing, average time
    strategy) of random single-layer transmissions in 24-PRB grids (DM-RS type 1)."""
    from pusch_chest_cases import random_case
    out = {}
    for i, (nrb, fd) in enumerate([(1, 2), (2, 2), (3, 2), (7, 2), (24, 2), (5, 1), (4, 0), (12, 2)]):
        cfg, grid, _ = random_case(rng, 24, nof_rb=nrb, dmrs_type2=0)
        ce, nv, rsrp, epre, ta, cfo = ref.pusch_chest(cfg, grid, 24, fd=fd)
        out[f"case{i}_cfg"] = np.array([cfg[k] for k in PUSCH_CHEST_KEYS] + [fd], np.int64)
        out[f"case{i}_scaling"] = np.float32(cfg["scaling"])
        out[f"case{i}_grid"], out[f"case{i}_ch_est"] = grid, ce
        out[f"case{i}_stats"] = np.stack([nv, rsrp, epre])
    np.savez_compressed(os.path.join(OUT, "pusch_chest.npz"), **out)


def gen_pusch_chest_cfo(ref, rng):
    """Reference DM-RS channel estimates with CFO estimation (compensated or not), time alignment and both time-domain
    strategies (average, interpolate), DM-RS type 1 with 2-4 DM-RS symbols (and one 1-symbol case per strategy), on
    received grids rotated by a carrier frequency offset and delayed: du_low's default configuration (filter, average,
    CFO compensation: du_low_config.h:51-69) and its alternatives."""
    from pusch_chest_cases import random_case
    out = {}
    masks = [(1 << 2) | (1 << 11), (1 << 2) | (1 << 7) | (1 << 11), (1 << 2) | (1 << 5) | (1 << 8) | (1 << 11),
             (1 << 3) | (1 << 9), 1 << 2]
    i = 0
    for td in (0, 1):
        for comp in (1, 0):
            for j, (nrb, fd) in enumerate([(4, 2), (24, 2), (1, 2), (7, 1), (52, 0)]):
                mask = masks[(j + td + comp) % len(masks)]
                cfg, grid, _ = random_case(rng, 64, nof_rb=nrb, dmrs_type2=0, dmrs_mask=mask,
                                           cfo_hz=float(rng.uniform(-1500, 1500)), delay=float(rng.uniform(-25, 25)))
                cfg["start_symbol"], cfg["nof_symbols"] = 0, 14
                ce, nv, rsrp, epre, ta, cfo = ref.pusch_chest(cfg, grid, 64, fd=fd, td=td, compensate_cfo=bool(comp))
                out[f"case{i}_cfg"] = np.array([cfg[k] for k in PUSCH_CHEST_KEYS] + [fd, td, comp], np.int64)
                out[f"case{i}_scaling"] = np.float32(cfg["scaling"])
                out[f"case{i}_grid"], out[f"case{i}_ch_est"] = grid, ce
                out[f"case{i}_stats"] = np.stack([nv, rsrp, epre, ta, cfo])
                i += 1
    np.savez_compressed(os.path.join(OUT, "pusch_chest_cfo.npz"), **out)


def gen_pusch_chest_low_papr(ref, rng):
    """Reference DM-RS channel estimates of transform-precoded PUSCH (low-PAPR DM-RS, n_RS_ID), 1..48 PRB (phase-table,
    length-30 and Zadoff-Chu sequences), du_low defaults (filter, average, CFO compensation) and interpolate."""
    from pusch_chest_cases import random_case
    out = {}
    for i, nrb in enumerate([1, 2, 3, 4, 5, 6, 10, 16, 24, 48]):
        td, comp, nid = i % 2, int(i % 3 != 2), int(rng.integers(0, 1008))
        cfg, grid, _ = random_case(rng, 64, nof_rb=nrb, dmrs_type2=0, dmrs_mask=(1 << 2) | (1 << 11),
                                   cfo_hz=float(rng.uniform(-1500, 1500)), delay=float(rng.uniform(-25, 25)),
                                   low_papr_id=nid)
        cfg["start_symbol"], cfg["nof_symbols"] = 0, 14
        ce, nv, rsrp, epre, ta, cfo = ref.pusch_chest(cfg, grid, 64, fd=2, td=td, compensate_cfo=bool(comp),
                                                      low_papr_id=nid)
        out[f"case{i}_cfg"] = np.array([cfg[k] for k in PUSCH_CHEST_KEYS] + [2, td, comp, nid], np.int64)
        out[f"case{i}_scaling"] = np.float32(cfg["scaling"])
        out[f"case{i}_grid"], out[f"case{i}_ch_est"] = grid, ce
        out[f"case{i}_stats"] = np.stack([nv, rsrp, epre, ta, cfo])
    np.savez_compressed(os.path.join(OUT, "pusch_chest_low_papr.npz"), **out)


PUSCH_CHEST_273_ROWS = (0, 2, 6, 11, 13)


def gen_pusch_chest_273(ref, rng):
    """Reference DM-RS channel estimates of configs[4]'s wideband jobs: one 273-PRB single-layer transmission (1638
    pilots per DM-RS symbol, the estimator's more-than-one-pilot-per-lane path) on 4 rx ports, DM-RS symbols 2 and 11,
    du_low defaults (filter, average, CFO compensation). Channels: the bench's synthetic test-mode channel (flat
    random unitary column + a phase ramp of up to 16 samples, bench.py / srsgpu/slot.py synthesize_uplink) at 26 and
    30 dB, and a frequency-selective delay-spread channel; plus a 160-PRB and a 272-PRB case off the band start. Only the
    DM-RS symbols of the grid are stored (the estimator reads nothing else) and estimate rows PUSCH_CHEST_273_ROWS."""
    import pusch_chest_oracle as C
    from pusch_chest_cases import random_case
    from pusch_demod_cases import bf16
    out = {}
    G, P = 273, 4
    nsc = 12 * G
    k = np.arange(nsc)
    mask = (1 << 2) | (1 << 11)
    ep = C.symbol_start_epochs(1)
    for i, (nrb, rb0, snr, kind) in enumerate([(273, 0, 26.0, "flat"), (273, 0, 30.0, "flat"), (273, 0, 26.0, "sel"),
                                               (160, 57, 22.0, "sel"), (272, 1, 30.0, "flat")]):
        cfg = dict(slot=int(rng.integers(0, 20)), scrambling_id=int(rng.integers(0, 1008)), n_scid=0, dmrs_type2=0,
                   scaling=float(10 ** (3 / 20)), dmrs_symbol_mask=mask, start_symbol=0, nof_symbols=14,
                   rb_start=rb0, nof_rb=nrb, nof_rx_ports=P)
        if kind == "flat":
            g = rng.normal(size=(P, P)) + 1j * rng.normal(size=(P, P))
            q, _ = np.linalg.qr(g)
            H = q[:, 0][:, None] * np.exp(2j * np.pi * k * rng.uniform() / 256)[None, :]
        else:
            H = np.zeros((P, nsc), np.complex128)
            for p in range(P):
                for _ in range(4):
                    H[p] += (rng.normal() + 1j * rng.normal()) / np.sqrt(8) * \
                        np.exp(-2j * np.pi * k * rng.uniform(0, 40) / 4096)
        x = (rng.choice([-1, 1], (14, nsc)) + 1j * rng.choice([-1, 1], (14, nsc))) / np.sqrt(2)
        sc = np.array([rb * 12 + 2 * j for rb in range(rb0, rb0 + nrb) for j in range(6)])
        for l in (2, 11):
            x[l, sc] = cfg["scaling"] * C.dmrs_sequence(cfg["slot"], l, cfg["scrambling_id"], 0, 0, rb0, nrb)
        cfo = float(rng.uniform(-300, 300))
        y = H[:, None, :] * x[None] * np.exp(2j * np.pi * cfo / 30000.0 * ep)[None, :, None]
        y = y + (rng.normal(size=y.shape) + 1j * rng.normal(size=y.shape)) * np.sqrt(10 ** (-snr / 10) / 2)
        grid = bf16(y)
        ce, nv, rsrp, epre, ta, cfo_hz = ref.pusch_chest(cfg, grid, G, fd=2, td=0, compensate_cfo=True)
        out[f"case{i}_cfg"] = np.array([cfg[k_] for k_ in PUSCH_CHEST_KEYS], np.int64)
        out[f"case{i}_scaling"] = np.float32(cfg["scaling"])
        out[f"case{i}_grid_dmrs"] = grid[:, [2, 11]]
        out[f"case{i}_ch_est_rows"] = ce[:, list(PUSCH_CHEST_273_ROWS)]
        out[f"case{i}_stats"] = np.stack([nv, rsrp, epre, ta, cfo_hz])
    np.savez_compressed(os.path.join(OUT, "pusch_chest_273.npz"), **out)


def gen_pdsch_dmrs(ref, rng):
    """Reference PDSCH DM-RS grids (dmrs_pdsch_processor_impl) of random configurations in 24-PRB grids."""
    from pdsch_dmrs_cases import random_config
    out = {}
    for i in range(10):
        cfg, w = random_config(rng, 24)
        out[f"case{i}_cfg"] = np.array([cfg[k] for k in PDSCH_DMRS_KEYS], np.int64)
        out[f"case{i}_amplitude"] = np.float32(cfg["amplitude"])
        out[f"case{i}_weights"] = w
        out[f"case{i}_grid"] = ref.dmrs_pdsch_map(cfg, w, 24)
    np.savez_compressed(os.path.join(OUT, "pdsch_dmrs.npz"), **out)


def gen_pdsch_dmrs_mask(ref, rng):
    """Reference PDSCH DM-RS grids over general CRB masks (config_t::rb_mask) in 51-PRB grids."""
    from pdsch_dmrs_cases import random_mask_config
    out = {}
    for i in range(8):
        cfg, w, mask = random_mask_config(rng, 51)
        out[f"case{i}_cfg"] = np.array([cfg[k] for k in PDSCH_DMRS_KEYS], np.int64)
        out[f"case{i}_amplitude"] = np.float32(cfg["amplitude"])
        out[f"case{i}_weights"] = w
        out[f"case{i}_crb_mask"] = mask
        out[f"case{i}_grid"] = ref.dmrs_pdsch_map(cfg, w, 51, crb_mask=mask)
    np.savez_compressed(os.path.join(OUT, "pdsch_dmrs_mask.npz"), **out)


PDSCH_DMRS_KEYS = ["slot", "scrambling_id", "n_scid", "dmrs_type2", "nof_layers", "nof_ports", "dmrs_symbol_mask",
                   "reference_point_k_rb", "rb_start", "nof_rb"]

PUSCH_CHEST_KEYS = ["slot", "scrambling_id", "n_scid", "dmrs_type2", "dmrs_symbol_mask", "start_symbol", "nof_symbols",
                    "rb_start", "nof_rb", "nof_rx_ports"]

PUSCH_DEMOD_KEYS = ["rnti", "n_id", "qm", "nof_layers", "nof_rx_ports", "start_symbol", "nof_symbols",
                    "dmrs_symbol_mask", "dmrs_type2", "nof_cdm_groups_without_data", "rb_start", "nof_rb"]


def gen_pdsch_mod_general(ref, rng):
    """General PDSCH allocations made by the reference (ref_pdsch_modulate_ex): VRB bitmaps non-interleaved /
    interleaved, reserved RE patterns, wideband or single-PRG precoding (multi-PRG: see
    test_pdsch_modulator_multi_prg_reference_defect), each with the reference's CRB mask."""
    from oracle_lib import pdsch_modulate_general
    from pdsch_mod_cases import random_general_config
    G = 32
    out = {}
    for i in range(10):
        cfg, nbits, w = random_general_config(rng, G, interleave=[0, 2, 4][i % 3], prg=[0, G][i % 2])
        cw = rng.integers(0, 256, (nbits + 7) // 8).astype(np.uint8)
        grid, crb = pdsch_modulate_general(ref.lib, cfg, w, cw, nbits, G)
        out[f"case{i}_cfg"] = np.array([cfg[k] for k in GENERAL_KEYS] + [nbits, G], np.int64)
        out[f"case{i}_scaling"] = np.float32(cfg["scaling"])
        out[f"case{i}_vrb"] = cfg["vrb_mask"]
        out[f"case{i}_res_crb"] = np.array([r[0] for r in cfg["reserved"]], np.uint8).reshape(-1, G)
        out[f"case{i}_res_masks"] = np.array([[r[1], r[2]] for r in cfg["reserved"]], np.int64).reshape(-1, 2)
        out[f"case{i}_w"] = w
        out[f"case{i}_prg_w"] = cfg["prg_weights"] if cfg["prg_size"] else np.zeros((0,), np.complex64)
        out[f"case{i}_cw"] = cw
        out[f"case{i}_grid"] = grid
        out[f"case{i}_crb"] = crb
    np.savez_compressed(os.path.join(OUT, "pdsch_mod_general.npz"), **out)


GENERAL_KEYS = ["rnti", "n_id", "qm", "nof_layers", "nof_ports", "bwp_start_rb", "bwp_size_rb", "start_symbol",
                "nof_symbols", "dmrs_symbol_mask", "dmrs_type2", "nof_cdm_groups_without_data", "interleave",
                "prg_size"]


def main():
    os.makedirs(OUT, exist_ok=True)
    ref = Reference()
    if len(sys.argv) > 1:  # regenerate only the named fixture sets, e.g. `python tools/gen_golden.py ofdm`
        for name in sys.argv[1:]:
            seed = {"ofdm": 16, "pusch_demod": 17, "pusch_chest": 18, "pdsch_dmrs": 19, "pusch_chest_cfo": 20,
                    "pdsch_mod_general": 21, "pdsch_dmrs_mask": 22, "pusch_demod_general": 23, "ulsch_demux": 24, "pusch_chest_low_papr": 25,
                    "pusch_chest_273": 26}[name]
            globals()["gen_" + name](ref, np.random.default_rng(seed))
        return
    gen_crc(ref, np.random.default_rng(10))
    gen_encoder(ref, np.random.default_rng(11))
    gen_decoder(ref, np.random.default_rng(12))
    gen_rate_matching(ref, np.random.default_rng(13))
    gen_pdsch_encoder(ref, np.random.default_rng(14))
    gen_pdsch_modulator(ref, np.random.default_rng(15))
    gen_ofdm(ref, np.random.default_rng(16))
    gen_pusch_demod(ref, np.random.default_rng(17))
    gen_pusch_chest(ref, np.random.default_rng(18))
    gen_pdsch_dmrs(ref, np.random.default_rng(19))
    gen_pusch_chest_cfo(ref, np.random.default_rng(20))
    gen_pdsch_mod_general(ref, np.random.default_rng(21))
    gen_pdsch_dmrs_mask(ref, np.random.default_rng(22))
    gen_pusch_demod_general(ref, np.random.default_rng(23))
    gen_ulsch_demux(ref, np.random.default_rng(24))
    gen_pusch_chest_low_papr(ref, np.random.default_rng(25))
    gen_pusch_chest_273(ref, np.random.default_rng(26))
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
