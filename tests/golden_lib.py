"""Iterators over the reference-generated fixtures in tests/golden/ (see tools/gen_golden.py)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BG_K = {1: 22, 2: 10}
BG_N_SHORT = {1: 66, 2: 50}


def _load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def crc_cases():
    d = _load("crc.npz")
    off = 0
    for poly, n, c in zip(d["poly"], d["lens"], d["crc"]):
        yield int(poly), d["bits"][off:off + n], int(c)
        off += n


def encoder_cases():
    d = _load("ldpc_encoder.npz")
    mo = co = 0
    for bg, Z in d["cfg"]:
        K, N = BG_K[bg] * Z, BG_N_SHORT[bg] * Z
        mb, cbb = (K + 7) // 8, (N + 7) // 8
        yield int(bg), int(Z), np.unpackbits(d["msg"][mo:mo + mb])[:K], np.unpackbits(d["cb"][co:co + cbb])[:N]
        mo += mb
        co += cbb


def decoder_cases():
    """Yields dict(bg, Z, impl (0 generic / 1 avx2), crc_poly (-1 none), nof_crc_bits, filler, max_iter, llr,
    iters (-1 = nullopt), bits)."""
    d = _load("ldpc_decoder.npz")
    lo = oo = 0
    for i, (bg, Z, impl, poly, nbits, filler, max_iter, n_llr) in enumerate(d["cfg"]):
        K = BG_K[bg] * Z
        ob = (K + 7) // 8
        yield dict(bg=int(bg), Z=int(Z), impl=int(impl), crc_poly=int(poly), nof_crc_bits=int(nbits),
                   filler=int(filler), max_iter=int(max_iter), llr=d["llr"][lo:lo + n_llr], iters=int(d["iters"][i]),
                   bits=np.unpackbits(d["out"][oo:oo + ob])[:K])
        lo += n_llr
        oo += ob


def rate_matching_cases():
    """Yields dict(bg, Z, rv, qm, Nref, filler, E, msg, rm_out, dm_llr, dm_init, dm_out[(new_data, impl)])."""
    d = _load("rate_matching.npz")
    mo = ro = lo = io = oo = 0
    for bg, Z, rv, qm, Nref, filler, E in d["cfg"]:
        K, N = BG_K[bg] * Z, BG_N_SHORT[bg] * Z
        mb, rb = (K + 7) // 8, (E + 7) // 8
        case = dict(bg=int(bg), Z=int(Z), rv=int(rv), qm=int(qm), Nref=int(Nref), filler=int(filler), E=int(E),
                    msg=np.unpackbits(d["msg"][mo:mo + mb])[:K], rm_out=np.unpackbits(d["rm_out"][ro:ro + rb])[:E],
                    dm_llr=d["dm_llr"][lo:lo + E], dm_init=d["dm_init"][io:io + N], dm_out={})
        for new_data in (1, 0):
            for impl in (0, 1):
                case["dm_out"][(new_data, impl)] = d["dm_out"][oo:oo + N]
                oo += N
        mo += mb
        ro += rb
        lo += E
        io += N
        yield case


def pdsch_encoder_cases():
    """Yields dict(bg, rv, qm, nof_layers, Nref, nof_ch_symbols, tb, cw (unpacked bits), meta (C x 4))."""
    d = _load("pdsch_encoder.npz")
    to = co = mo = 0
    for bg, rv, qm, layers, Nref, nsym, tb_bytes, ncb in d["cfg"]:
        G = nsym * qm
        cb = (G + 7) // 8
        yield dict(bg=int(bg), rv=int(rv), qm=int(qm), nof_layers=int(layers), Nref=int(Nref),
                   nof_ch_symbols=int(nsym), tb=d["tb"][to:to + tb_bytes], cw=np.unpackbits(d["cw"][co:co + cb])[:G],
                   meta=d["meta"][mo:mo + ncb])
        to += tb_bytes
        co += cb
        mo += ncb


def pdsch_modulator_cases():
    """Yields (cfg dict, nof_bits, grid_nof_prb, weights (P x L complex64), packed codeword, grid uint16
    (P, 14, 12 * grid_nof_prb, 2)) made by the reference's pdsch_modulator_impl."""
    from oracle_lib import PDSCH_MOD_KEYS
    d = _load("pdsch_modulator.npz")
    wo = co = go = 0
    for row, scaling in zip(d["cfg"], d["scaling"]):
        cfg = {k: int(v) for k, v in zip(PDSCH_MOD_KEYS[:-1], row[:-2])}
        cfg["scaling"] = float(scaling)
        nbits, grid_prb = int(row[-2]), int(row[-1])
        P, L = cfg["nof_ports"], cfg["nof_layers"]
        nw, nc, ng = P * L, (nbits + 7) // 8, P * 14 * 12 * grid_prb * 2
        yield (cfg, nbits, grid_prb, d["weights"][wo:wo + nw].reshape(P, L), d["cw"][co:co + nc],
               d["grid"][go:go + ng].reshape(P, 14, 12 * grid_prb, 2))
        wo += nw
        co += nc
        go += ng


def ofdm_cases():
    """Yields (case tuple of ofdm_cases.CASES, input bf16 grid (P, nsymb, nsc, 2), reference-modulated samples
    (P, slot_size) complex64, reference-demodulated bf16 grid of those samples with scale 1 / (scale * N))."""
    from ofdm_cases import CASES
    d = _load("ofdm.npz")
    i = 0
    while f"case{i}_params" in d:
        c = int(d[f"case{i}_params"][0])
        yield CASES[c], d[f"case{i}_grid"], d[f"case{i}_samples"], d[f"case{i}_demod"]
        i += 1


PUSCH_DEMOD_KEYS = ["rnti", "n_id", "qm", "nof_layers", "nof_rx_ports", "start_symbol", "nof_symbols",
                    "dmrs_symbol_mask", "dmrs_type2", "nof_cdm_groups_without_data", "rb_start", "nof_rb"]


def pusch_demod_cases():
    """Yields (cfg dict, mmse flag, grid (P, 14, 288, 2) bf16, ch_est (L, P, 14, 288, 2) bf16, noise_var (P,),
    reference LLRs) made by the reference's pusch_demodulator_impl (24-PRB grids)."""
    d = _load("pusch_demod.npz")
    i = 0
    while f"case{i}_cfg" in d:
        row = d[f"case{i}_cfg"]
        cfg = {k: int(v) for k, v in zip(PUSCH_DEMOD_KEYS, row[:-1])}
        yield (cfg, bool(row[-1]), d[f"case{i}_grid"], d[f"case{i}_ch_est"], d[f"case{i}_noise_var"],
               d[f"case{i}_llr"])
        i += 1


def pusch_demod_general_cases():
    """Yields (cfg dict, transform precoding flag, CRB mask or None, grid (P, 14, 384, 2) bf16, ch_est, noise_var,
    reference LLRs, reference stats (15, 2): per-symbol and end (SINR dB, EVM), NaN when absent) made by
    pusch_demodulator_impl with the EVM calculator, post-equalization SINR, CRB masks and transform precoding
    (32-PRB grids)."""
    d = _load("pusch_demod_general.npz")
    i = 0
    while f"case{i}_cfg" in d:
        row = d[f"case{i}_cfg"]
        cfg = {k: int(v) for k, v in zip(PUSCH_DEMOD_KEYS, row[:-1])}
        crb = d[f"case{i}_crb"]
        yield (cfg, bool(row[-1]), crb if crb.size else None, d[f"case{i}_grid"], d[f"case{i}_ch_est"],
               d[f"case{i}_noise_var"], d[f"case{i}_llr"], d[f"case{i}_stats"])
        i += 1


def demapper_cases():
    """Yields (qm, symbols complex64, noise variances, reference LLRs) made by demodulation_mapper_impl."""
    d = _load("pusch_demod.npz")
    for qm in (2, 4, 6, 8):
        yield qm, d[f"demap{qm}_symbols"], d[f"demap{qm}_noise_var"], d[f"demap{qm}_llr"]


PUSCH_CHEST_KEYS = ["slot", "scrambling_id", "n_scid", "dmrs_type2", "dmrs_symbol_mask", "start_symbol", "nof_symbols",
                    "rb_start", "nof_rb", "nof_rx_ports"]


def pusch_chest_cases():
    """Yields (cfg dict, fd strategy (0 none, 1 mean, 2 filter), grid (P, 14, 288, 2) bf16, reference estimates
    (P, 14, 288, 2) bf16 (valid on the allocation only), [noise_var, rsrp, epre] (3, P)) made by
    dmrs_pusch_estimator_impl."""
    d = _load("pusch_chest.npz")
    i = 0
    while f"case{i}_cfg" in d:
        row = d[f"case{i}_cfg"]
        cfg = {k: int(v) for k, v in zip(PUSCH_CHEST_KEYS, row[:-1])}
        cfg["scaling"] = float(d[f"case{i}_scaling"])
        yield cfg, int(row[-1]), d[f"case{i}_grid"], d[f"case{i}_ch_est"], d[f"case{i}_stats"]
        i += 1


def pusch_chest_cfo_cases():
    """Yields (cfg dict, fd, td (0 average, 1 interpolate), compensate_cfo, grid (P, 14, 768, 2) bf16, reference
    estimates, [noise_var, rsrp, epre, ta_s, cfo_hz] (5, P)) made by dmrs_pusch_estimator_impl on 64-PRB grids."""
    d = _load("pusch_chest_cfo.npz")
    i = 0
    while f"case{i}_cfg" in d:
        row = d[f"case{i}_cfg"]
        cfg = {k: int(v) for k, v in zip(PUSCH_CHEST_KEYS, row[:-3])}
        cfg["scaling"] = float(d[f"case{i}_scaling"])
        yield (cfg, int(row[-3]), int(row[-2]), int(row[-1]), d[f"case{i}_grid"], d[f"case{i}_ch_est"],
               d[f"case{i}_stats"])
        i += 1


def pusch_chest_low_papr_cases():
    """Yields (cfg dict, fd, td, compensate_cfo, n_RS_ID, grid (P, 14, 768, 2) bf16, reference estimates, [noise_var,
    rsrp, epre, ta_s, cfo_hz] (5, P)) made by dmrs_pusch_estimator_impl with low-PAPR DM-RS (64-PRB grids)."""
    d = _load("pusch_chest_low_papr.npz")
    i = 0
    while f"case{i}_cfg" in d:
        row = d[f"case{i}_cfg"]
        cfg = {k: int(v) for k, v in zip(PUSCH_CHEST_KEYS, row[:-4])}
        cfg["scaling"] = float(d[f"case{i}_scaling"])
        yield (cfg, int(row[-4]), int(row[-3]), int(row[-2]), int(row[-1]), d[f"case{i}_grid"],
               d[f"case{i}_ch_est"], d[f"case{i}_stats"])
        i += 1


PUSCH_CHEST_273_ROWS = (0, 2, 6, 11, 13)


def pusch_chest_273_cases():
    """Yields (cfg dict, grid (P, 14, 3276, 2) bf16 with only DM-RS symbols 2 and 11 filled, reference estimate rows
    PUSCH_CHEST_273_ROWS (P, 5, 3276, 2), [noise_var, rsrp, epre, ta_s, cfo_hz] (5, P)) made by
    dmrs_pusch_estimator_impl on configs[4]'s wideband (160-273 PRB) jobs: filter, average, CFO compensation."""
    d = _load("pusch_chest_273.npz")
    i = 0
    while f"case{i}_cfg" in d:
        cfg = {k: int(v) for k, v in zip(PUSCH_CHEST_KEYS, d[f"case{i}_cfg"])}
        cfg["scaling"] = float(d[f"case{i}_scaling"])
        gd = d[f"case{i}_grid_dmrs"]
        grid = np.zeros((gd.shape[0], 14) + gd.shape[2:], np.uint16)
        grid[:, [2, 11]] = gd
        yield cfg, grid, d[f"case{i}_ch_est_rows"], d[f"case{i}_stats"]
        i += 1


PDSCH_DMRS_KEYS = ["slot", "scrambling_id", "n_scid", "dmrs_type2", "nof_layers", "nof_ports", "dmrs_symbol_mask",
                   "reference_point_k_rb", "rb_start", "nof_rb"]


def pdsch_dmrs_cases():
    """Yields (cfg dict, weights (P, L) complex64, reference grid (P, 14, 288, 2) bf16) made by
    dmrs_pdsch_processor_impl (24-PRB grids)."""
    d = _load("pdsch_dmrs.npz")
    i = 0
    while f"case{i}_cfg" in d:
        cfg = {k: int(v) for k, v in zip(PDSCH_DMRS_KEYS, d[f"case{i}_cfg"])}
        cfg["amplitude"] = float(d[f"case{i}_amplitude"])
        yield cfg, d[f"case{i}_weights"], d[f"case{i}_grid"]
        i += 1


def pdsch_dmrs_mask_cases():
    """Yields (cfg dict, weights (P, L) complex64, CRB mask (51,) uint8, reference grid (P, 14, 612, 2) bf16) made by
    dmrs_pdsch_processor_impl with general rb_mask allocations (51-PRB grids)."""
    d = _load("pdsch_dmrs_mask.npz")
    i = 0
    while f"case{i}_cfg" in d:
        cfg = {k: int(v) for k, v in zip(PDSCH_DMRS_KEYS, d[f"case{i}_cfg"])}
        cfg["amplitude"] = float(d[f"case{i}_amplitude"])
        yield cfg, d[f"case{i}_weights"], d[f"case{i}_crb_mask"], d[f"case{i}_grid"]
        i += 1


GENERAL_KEYS = ["rnti", "n_id", "qm", "nof_layers", "nof_ports", "bwp_start_rb", "bwp_size_rb", "start_symbol",
                "nof_symbols", "dmrs_symbol_mask", "dmrs_type2", "nof_cdm_groups_without_data", "interleave",
                "prg_size"]


def pdsch_mod_general_cases():
    """Yields (cfg dict with vrb_mask / interleave / reserved / prg_size / prg_weights, nof_bits, grid_nof_prb,
    weights (P x L complex64), packed codeword, reference grid (P, 14, nsc, 2) uint16, reference CRB mask) made by the
    reference's pdsch_modulator_impl with general allocations (tools/gen_golden.py gen_pdsch_mod_general)."""
    d = _load("pdsch_mod_general.npz")
    i = 0
    while f"case{i}_cfg" in d:
        row = d[f"case{i}_cfg"]
        cfg = {k: int(v) for k, v in zip(GENERAL_KEYS, row[:-2])}
        nbits, G = int(row[-2]), int(row[-1])
        cfg.update(rb_start=0, nof_rb=0, scaling=float(d[f"case{i}_scaling"]), vrb_mask=d[f"case{i}_vrb"],
                   reserved=[(c, int(m[0]), int(m[1])) for c, m in zip(d[f"case{i}_res_crb"], d[f"case{i}_res_masks"])],
                   prg_weights=d[f"case{i}_prg_w"] if cfg["prg_size"] else None)
        yield cfg, nbits, G, d[f"case{i}_w"], d[f"case{i}_cw"], d[f"case{i}_grid"], d[f"case{i}_crb"]
        i += 1


ULSCH_DEMUX_KEYS = ["qm", "nof_layers", "nof_prb", "start_symbol", "nof_symbols", "dmrs_symbol_mask", "dmrs_type2",
                    "nof_cdm_groups_without_data", "nof_harq_ack_rvd", "nof_harq_ack_bits", "nof_enc_harq_ack_bits",
                    "nof_csi_part1_bits", "nof_enc_csi_part1_bits"]


def ulsch_demux_cases():
    """Yields (cfg dict, CSI-2 bits, CSI-2 encoded bits, c_init, codeword LLRs int8, reference outputs dict sch / harq /
    csi1 / csi2) made by the reference's ulsch_demultiplex_impl."""
    d = _load("ulsch_demux.npz")
    i = 0
    while f"case{i}_cfg" in d:
        row = d[f"case{i}_cfg"]
        cfg = {k: int(v) for k, v in zip(ULSCH_DEMUX_KEYS, row[:-3])}
        yield (cfg, int(row[-3]), int(row[-2]), int(row[-1]), d[f"case{i}_llrs"],
               {k: d[f"case{i}_{k}"] for k in ("sch", "harq", "csi1", "csi2")})
        i += 1
