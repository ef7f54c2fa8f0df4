"""Pins the CPU oracle (and the host SCH logic) against the fixtures the reference produced (tests/golden/, made by
tools/gen_golden.py from the reference built from its own sources). Runs everywhere, no reference tree needed."""
import numpy as np
import pytest

import golden_lib as G
from oracle_lib import Oracle
from chain_lib import oracle_pdsch_encode


@pytest.fixture(scope="module")
def orc():
    return Oracle()


def test_crc_golden(orc):
    n = 0
    for poly, bits, want in G.crc_cases():
        assert orc.crc_bits(poly, bits) == want
        n += 1
    assert n == 30


def test_encoder_golden(orc):
    for bg, Z, msg, cb in G.encoder_cases():
        assert np.array_equal(orc.ldpc_encode(bg, Z, msg), cb), (bg, Z)


def test_decoder_golden(orc):
    nsucc = nfail = 0
    for c in G.decoder_cases():
        r, bits = orc.ldpc_decode(c["impl"], c["bg"], c["Z"], c["llr"], nof_crc_bits=c["nof_crc_bits"],
                                  nof_filler=c["filler"], crc_poly=c["crc_poly"], max_iter=c["max_iter"], scaling=0.8)
        assert r == c["iters"], c["Z"]
        assert np.array_equal(bits, c["bits"])
        nsucc += r >= 0
        nfail += r < 0
    assert nsucc > 20 and nfail > 20


def test_rate_matching_golden(orc):
    for c in G.rate_matching_cases():
        cb = orc.ldpc_encode(c["bg"], c["Z"], c["msg"])
        out = orc.rate_match(c["bg"], c["Z"], c["rv"], c["qm"], c["Nref"], c["filler"], cb, c["E"])
        assert np.array_equal(out, c["rm_out"])
        for (new_data, impl), want in c["dm_out"].items():
            got = orc.rate_dematch(impl, c["bg"], c["Z"], c["rv"], c["qm"], c["Nref"], c["filler"], new_data,
                                   c["dm_llr"], c["dm_init"])
            assert np.array_equal(got, want), (c["Z"], c["rv"], new_data, impl)


def test_pdsch_encoder_golden(orc):
    n = 0
    for c in G.pdsch_encoder_cases():
        cw, seg, _ = oracle_pdsch_encode(orc, c["tb"], c["bg"], c["rv"], c["qm"], c["nof_layers"], c["Nref"],
                                         c["nof_ch_symbols"])
        assert seg.nof_segments == c["meta"].shape[0]
        assert np.array_equal(cw, c["cw"])
        n += 1
    assert n == 14


def test_pdsch_modulator_golden(orc):
    n = 0
    for cfg, nbits, grid_prb, w, cw, grid in G.pdsch_modulator_cases():
        assert np.array_equal(orc.pdsch_modulate(cfg, w, cw, nbits, grid_prb), grid), cfg
        n += 1
    assert n == 12


def test_pdsch_mod_general_golden(orc):
    """General allocations (VRB bitmaps, interleaving, reserved REs, single-PRG precoding): the test-side CRB mapping
    and the product's host mapping reproduce the reference's CRB masks, and the oracle reproduces its grids."""
    import srsgpu.alloc as A
    from oracle_lib import pdsch_modulate_general
    from pdsch_mod_cases import crb_mask_test_side
    n = 0
    for cfg, nbits, grid_prb, w, cw, grid, crb in G.pdsch_mod_general_cases():
        assert np.array_equal(crb_mask_test_side(cfg, grid_prb), crb)
        il = cfg["interleave"]
        vtp = A.interleaved_other(cfg["bwp_start_rb"], cfg["bwp_size_rb"], il) if il else None
        assert np.array_equal(A.vrb_to_crb_mask(cfg["vrb_mask"], cfg["bwp_start_rb"], cfg["bwp_size_rb"], grid_prb,
                                                vtp), crb)
        got, _ = pdsch_modulate_general(orc.lib, cfg, w, cw, nbits, grid_prb, crb_mask=crb)
        assert np.array_equal(got, grid), cfg
        n += 1
    assert n == 10


def test_ofdm_golden():
    """The numpy OFDM restatement against the reference modulator's samples and demodulator's grids."""
    import ofdm_oracle as O
    from ofdm_cases import bf16_close, rel_err
    n = 0
    for (mu, rb, N, ext, scale, fc, slot, woff), grid, samples, demod in G.ofdm_cases():
        got = O.modulate(grid, mu, rb, N, ext, scale, fc, slot)
        assert rel_err(got, samples) < 2e-5
        g2 = O.complex_to_bf16(O.demodulate(samples.astype(np.complex128), mu, rb, N, ext, 1.0 / (scale * N), fc,
                                            slot, woff))
        ok, frac = bf16_close(g2, demod)
        assert ok and frac < 0.02, frac
        n += 1
    assert n == 5


def test_pusch_demod_golden():
    """The numpy PUSCH demodulator / demapper restatement against the reference's LLRs (within one quantisation step
    on a small fraction: the reference's AVX2 equalizer uses an approximate reciprocal)."""
    import pusch_demod_oracle as D
    from pusch_demod_cases import from_bf16
    n = 0
    for cfg, mmse, grid, H, nv, want in G.pusch_demod_cases():
        got = D.demodulate(cfg, from_bf16(grid), from_bf16(H), nv, mmse).astype(np.int16)
        d = np.abs(got - want.astype(np.int16))
        assert got.size == want.size and d.max() <= 1 and np.mean(d > 0) < 0.05, (cfg, d.max(), np.mean(d > 0))
        n += 1
    assert n == 9
    for qm, x, nv, want in G.demapper_cases():
        d = np.abs(D.demap(x, nv, qm).astype(np.int16) - want.astype(np.int16))
        assert d.max() <= 1 and np.mean(d > 0) < 0.01, qm


def test_pusch_chest_golden():
    """The numpy DM-RS channel estimator restatement against the reference's estimates (allocation only) and noise
    variance / RSRP / EPRE."""
    import pusch_chest_oracle as C
    from ofdm_oracle import bf16_to_complex
    n = 0
    for cfg, fd, grid, ce, stats in G.pusch_chest_cases():
        ch, nv, rsrp, epre, _ = C.estimate(cfg, bf16_to_complex(grid), ["none", "mean", "filter"][fd])
        l0, l1 = cfg["start_symbol"], cfg["start_symbol"] + cfg["nof_symbols"]
        k0, k1 = cfg["rb_start"] * 12, (cfg["rb_start"] + cfg["nof_rb"]) * 12
        want = bf16_to_complex(ce)[:, l0:l1, k0:k1]
        got = ch[:, l0:l1, k0:k1]
        assert np.max(np.abs(got - want)) < 1e-2 * np.sqrt(np.mean(np.abs(want) ** 2))
        np.testing.assert_allclose(np.stack([nv, rsrp, epre]), stats, rtol=1e-3)
        n += 1
    assert n == 8


# Stated tolerances of the CFO / TA / time-strategy fixtures (reference float32 + bf16 estimates vs the float64
# restatement): estimates within CHEST_CFO_TOL[td] x RMS channel ("interpolate" extrapolates past the DM-RS symbols,
# amplifying the reference's bf16 / float rounding), noise variance / RSRP / EPRE 1e-3 relative, CFO within 0.05 Hz,
# time alignment within 2 Tc (the reference rounds to Tc).
CHEST_CFO_TOL = {0: 1.5e-2, 1: 2.5e-2}
T_C = 1.0 / (480000 * 4096)


def test_pusch_chest_cfo_golden():
    """The restatement against the reference's estimates with CFO estimation / compensation, time alignment and the
    average / interpolate time strategies (tests/golden/pusch_chest_cfo.npz)."""
    import pusch_chest_oracle as C
    from ofdm_oracle import bf16_to_complex
    n = 0
    for cfg, fd, td, comp, grid, ce, stats in G.pusch_chest_cfo_cases():
        ch, nv, rsrp, epre, ex = C.estimate(cfg, bf16_to_complex(grid), ["none", "mean", "filter"][fd],
                                            ["average", "interpolate"][td], bool(comp))
        k0, k1 = cfg["rb_start"] * 12, (cfg["rb_start"] + cfg["nof_rb"]) * 12
        want = bf16_to_complex(ce)[:, :, k0:k1]
        got = ch[:, :, k0:k1]
        assert np.max(np.abs(got - want)) < CHEST_CFO_TOL[td] * np.sqrt(np.mean(np.abs(want) ** 2)), (n, cfg)
        np.testing.assert_allclose(np.stack([nv, rsrp, epre]), stats[:3], rtol=1e-3)
        np.testing.assert_allclose(ex["ta_s"], stats[3], atol=2 * T_C)
        np.testing.assert_allclose(ex["cfo_hz"], stats[4], atol=0.05)  # NaN == NaN (one DM-RS symbol)
        n += 1
    assert n == 20


def test_pusch_chest_low_papr_golden():
    """The restatement against the reference's estimates of transform-precoded PUSCH (low-PAPR DM-RS)."""
    import pusch_chest_oracle as C
    from ofdm_oracle import bf16_to_complex
    n = 0
    for cfg, fd, td, comp, nid, grid, ce, stats in G.pusch_chest_low_papr_cases():
        ch, nv, rsrp, epre, ex = C.estimate(cfg, bf16_to_complex(grid), ["none", "mean", "filter"][fd],
                                            ["average", "interpolate"][td], bool(comp), low_papr_id=nid)
        k0, k1 = cfg["rb_start"] * 12, (cfg["rb_start"] + cfg["nof_rb"]) * 12
        want = bf16_to_complex(ce)[:, :, k0:k1]
        got = ch[:, :, k0:k1]
        assert np.max(np.abs(got - want)) < CHEST_CFO_TOL[td] * np.sqrt(np.mean(np.abs(want) ** 2)), (n, cfg)
        np.testing.assert_allclose(np.stack([nv, rsrp, epre]), stats[:3], rtol=1e-3)
        np.testing.assert_allclose(ex["ta_s"], stats[3], atol=2 * T_C)
        np.testing.assert_allclose(ex["cfo_hz"], stats[4], atol=0.05)
        n += 1
    assert n == 10


def test_pusch_chest_273_golden():
    """The restatement against the reference's estimates of configs[4]'s wideband jobs (160-273 PRB, 1638 pilots per
    DM-RS symbol): du_low defaults (filter, average, CFO compensation), tests/golden/pusch_chest_273.npz."""
    import pusch_chest_oracle as C
    from ofdm_oracle import bf16_to_complex
    n = 0
    rows = list(G.PUSCH_CHEST_273_ROWS)
    for cfg, grid, ce_rows, stats in G.pusch_chest_273_cases():
        ch, nv, rsrp, epre, ex = C.estimate(cfg, bf16_to_complex(grid), "filter", "average", True)
        k0, k1 = cfg["rb_start"] * 12, (cfg["rb_start"] + cfg["nof_rb"]) * 12
        want = bf16_to_complex(ce_rows)[:, :, k0:k1]
        got = ch[:, rows, k0:k1]
        assert np.max(np.abs(got - want)) < CHEST_CFO_TOL[0] * np.sqrt(np.mean(np.abs(want) ** 2)), (n, cfg)
        np.testing.assert_allclose(np.stack([nv, rsrp, epre]), stats[:3], rtol=1e-3)
        np.testing.assert_allclose(ex["ta_s"], stats[3], atol=2 * T_C)
        np.testing.assert_allclose(ex["cfo_hz"], stats[4], atol=0.05)
        n += 1
    assert n == 5


def test_pdsch_dmrs_golden():
    """The PDSCH DM-RS restatement bit-exact against the reference's grids."""
    import pdsch_dmrs_oracle as M
    n = 0
    for cfg, w, grid in G.pdsch_dmrs_cases():
        assert np.array_equal(M.dmrs_map(cfg, w, 24), grid), cfg
        n += 1
    assert n == 10


def test_pdsch_dmrs_crb_mask_golden():
    """The PDSCH DM-RS restatement over general CRB masks bit-exact against the reference's grids."""
    import pdsch_dmrs_oracle as M
    n = 0
    for cfg, w, mask, grid in G.pdsch_dmrs_mask_cases():
        assert np.array_equal(M.dmrs_map(cfg, w, 51, crb_mask=mask), grid), cfg
        n += 1
    assert n == 8


def test_pusch_demod_general_golden():
    """The demodulator restatement with CRB masks, transform precoding and the post-equalization statistics against
    the reference's LLRs (within one step on < 5 %), EVM (1e-2 relative per symbol: one hard decision flipped by the
    reference's approximate reciprocal moves a small symbol's EVM by ~0.5 %; 5e-3 for the total) and SINR (5e-3
    dB)."""
    import pusch_demod_oracle as D
    from pusch_demod_cases import from_bf16
    n = 0
    for cfg, tp, crb, grid, H, nv, want, wstats in G.pusch_demod_general_cases():
        got, gstats = D.demodulate_ex(cfg, from_bf16(grid), from_bf16(H), nv, crb_mask=crb, transform_precoding=tp)
        d = np.abs(got.astype(np.int16) - want.astype(np.int16))
        assert got.size == want.size and d.max() <= 1 and np.mean(d > 0) < 0.05, cfg
        assert np.array_equal(np.isnan(gstats), np.isnan(wstats))
        ok = ~np.isnan(wstats)
        np.testing.assert_allclose(gstats[:14, 1][ok[:14, 1]], wstats[:14, 1][ok[:14, 1]], rtol=1e-2)
        np.testing.assert_allclose(gstats[14, 1], wstats[14, 1], rtol=5e-3)
        # Two-layer ZF: the near-singular REs' noise variances dominate the mean and their 2 x 2 inverse is sensitive
        # to the rounding order (the reference: AVX2 with an approximate reciprocal), so 0.1 dB there.
        np.testing.assert_allclose(gstats[:, 0][ok[:, 0]], wstats[:, 0][ok[:, 0]],
                                   atol=5e-3 if cfg["nof_layers"] == 1 else 0.1)
        n += 1
    assert n == 8


def test_ulsch_demux_golden():
    """The UL-SCH demultiplexer restatement bit-exact against the reference's outputs."""
    import ulsch_demux_oracle as U
    n = 0
    for cfg, c2b, c2e, c_init, llrs, want in G.ulsch_demux_cases():
        got = U.demultiplex(cfg, llrs, c_init, c2b, c2e)
        for k in ("sch", "harq", "csi1", "csi2"):
            assert np.array_equal(got[k], want[k]), (k, cfg)
        n += 1
    assert n == 12
