"""GPU parity of the PUSCH demodulator (equalization + soft demapping + descrambling; srsgpu_pusch_demodulator_plan
through the C ABI) against the reference's own LLRs (tests/golden/pusch_demod.npz, made by pusch_demodulator_impl)
and the numpy restatement (oracle/pusch_demod_oracle.py).

Tolerances (soft LLRs, floating point): for the reference's paths (ZF 1 x N, ZF 2 x N, MMSE with one layer) every
LLR equal or one quantisation step (20 / 120) apart, < 5 % differing (the reference's AVX2 equalizer uses an
approximate reciprocal; the GPU divides exactly). For the multi-layer MMSE extension (float32
Cholesky on the GPU vs float64 numpy): >= 99 % of the LLRs within one step and the hard decisions (signs) of >= 99.5 % equal."""
import numpy as np
import pytest

import golden_lib as G
import pusch_demod_oracle as D
from pusch_demod_cases import from_bf16, random_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import srsgpu
    return srsgpu.Context(0)


def to_demod(cfg, mmse=False):
    import srsgpu
    return srsgpu.PuschDemodulation(
        rnti=cfg["rnti"], n_id=cfg["n_id"], modulation_order=cfg["qm"], nof_tx_layers=cfg["nof_layers"],
        nof_rx_ports=cfg["nof_rx_ports"], start_symbol=cfg["start_symbol"], nof_symbols=cfg["nof_symbols"],
        dmrs_symbol_mask=cfg["dmrs_symbol_mask"], dmrs_type=2 if cfg["dmrs_type2"] else 1,
        nof_cdm_groups_without_data=cfg["nof_cdm_groups_without_data"], rb_start=cfg["rb_start"],
        nof_rb=cfg["nof_rb"], equalizer=srsgpu.EQ_MMSE if mmse else srsgpu.EQ_ZF)


def pad_slot(grid, H, nv, Pg=4):
    """One slot's buffers in the plan layout: grid (Pg, 14, nsc, 2), estimates (4, Pg, 14, nsc, 2), noise (4,)."""
    P, L = grid.shape[0], H.shape[0]
    g = np.zeros((Pg,) + grid.shape[1:], np.uint16)
    g[:P] = grid
    h = np.zeros((4, Pg) + H.shape[2:], np.uint16)
    h[:L, :P] = H
    n = np.zeros(4, np.float32)
    n[:P] = nv
    return g, h, n


def close(got, want, frac=0.05):
    d = np.abs(got.astype(np.int16) - want.astype(np.int16))
    return d.max() <= 1 and np.mean(d > 0) < frac, (int(d.max()), float(np.mean(d > 0)))


def test_pusch_demod_golden(ctx):
    """Every reference-made case, all in ONE plan (one slot each)."""
    import srsgpu
    cases = list(G.pusch_demod_cases())
    grids, hs, nvs, demods = [], [], [], []
    for cfg, mmse, grid, H, nv, _ in cases:
        g, h, n = pad_slot(grid, H, nv)
        grids.append(g)
        hs.append(h)
        nvs.append(n)
        demods.append(to_demod(cfg, mmse))
    got = srsgpu.PuschDemodulator(ctx, 24, 4).demodulate_batch(np.stack(grids), np.stack(hs), np.stack(nvs), demods,
                                                               list(range(len(cases))))
    for (cfg, mmse, _, _, _, want), llr in zip(cases, got):
        ok, stats = close(llr, want)
        assert llr.size == want.size and ok, (cfg, stats)


@pytest.mark.parametrize("qm", [2, 4, 6, 8])
def test_pusch_demod_demapper_golden(ctx, qm):
    """The demapper through the whole kernel: one layer, one port, unit channel (the equalizer passes the symbol
    through with nvar = the port's noise variance), the reference demapper vectors' symbols, against the oracle demapper
    (itself pinned to those vectors) with the descrambling applied."""
    import srsgpu
    for q, x, nv, want in G.demapper_cases():
        if q != qm:
            continue
        n = 3900  # 25 PRB x 13 symbols x 12 REs, one DM-RS symbol without data
        cfg = dict(rnti=0, n_id=0, qm=qm, nof_layers=1, nof_rx_ports=1, start_symbol=0, nof_symbols=14,
                   dmrs_symbol_mask=1 << 2, dmrs_type2=0, nof_cdm_groups_without_data=2, rb_start=0, nof_rb=25)
        res = D.data_res(0, 14, 1 << 2, 0, 2, 0, 25)
        assert len(res) == n
        grid = np.zeros((4, 14, 300, 2), np.uint16)
        H = np.zeros((4, 4, 14, 300, 2), np.uint16)
        # The ZF output is y conj(h) / |h|^2 with nvar = nv: feed y = x (as bf16) and h = 1.
        from pusch_demod_cases import bf16
        xs = x[:n]
        for i, (l, k) in enumerate(res):
            grid[0, l, k] = bf16(np.array([xs[i]]))[0]
        H[0, 0, :, :, 0] = 0x3F80  # 1.0
        nvar = np.array([0.1, 0, 0, 0], np.float32)
        got = srsgpu.PuschDemodulator(ctx, 25, 4).demodulate_batch(grid[None], H[None], nvar[None],
                                                                   [to_demod(cfg)], [0])[0]
        xq = from_bf16(bf16(xs))
        ref_llr = D.demap(xq, np.full(n, 0.1, np.float32), qm).astype(np.int16)
        c = D.gold_sequence(0, ref_llr.size)
        want2 = np.where(c == 1, -ref_llr, ref_llr)
        ok, stats = close(got, want2, frac=0.001)
        assert ok, stats


def test_pusch_demod_random_batch(ctx):
    """60 random transmissions (1-2 layers, 1-4 ports, ZF / MMSE, every modulation, random DM-RS patterns), each in
    its own 40-PRB slot, in ONE plan, against the oracle."""
    import srsgpu
    rng = np.random.default_rng(42)
    prb = 40
    grids, hs, nvs, demods, want = [], [], [], [], []
    for t in range(60):
        cfg, grid, H, nv = random_case(rng, prb)
        mmse = bool(t % 4 == 3 and cfg["nof_layers"] == 1)
        g, h, n = pad_slot(grid, H, nv)
        grids.append(g)
        hs.append(h)
        nvs.append(n)
        demods.append(to_demod(cfg, mmse))
        want.append(D.demodulate(cfg, from_bf16(grid), from_bf16(H), nv, mmse))
    got = srsgpu.PuschDemodulator(ctx, prb, 4).demodulate_batch(np.stack(grids), np.stack(hs), np.stack(nvs), demods,
                                                                list(range(60)))
    for i, (a, b) in enumerate(zip(got, want)):
        ok, stats = close(a, b)
        assert a.size == b.size and ok, (i, demods[i], stats)


@pytest.mark.parametrize("L", [2, 3, 4])
def test_pusch_demod_mmse_multilayer(ctx, L):
    """MMSE with 2-4 layers over 4 ports (extension beyond the open-source reference) against float64 numpy MMSE."""
    import srsgpu
    rng = np.random.default_rng(50 + L)
    cfg, grid, H, nv = random_case(rng, 52, nof_layers=L, nof_rx_ports=4, snr_db=25)
    want = D.demodulate(cfg, from_bf16(grid), from_bf16(H), nv, mmse=True).astype(np.int16)
    g, h, n = pad_slot(grid, H, nv)
    got = srsgpu.PuschDemodulator(ctx, 52, 4).demodulate_batch(g[None], h[None], n[None], [to_demod(cfg, True)],
                                                               [0])[0].astype(np.int16)
    d = np.abs(got - want)
    assert np.mean(d <= 1) >= 0.99, np.mean(d <= 1)
    assert np.mean(np.sign(got) == np.sign(want)) >= 0.995


def test_pusch_demod_rejects_invalid(ctx):
    import srsgpu
    rng = np.random.default_rng(1)
    cfg, *_ = random_case(rng, 24, nof_layers=2, nof_rx_ports=2)
    for bad in [dict(nof_rx_ports=3), dict(qm=3), dict(rb_start=20, nof_rb=10), dict(nof_layers=3, nof_rx_ports=2)]:
        arr, _, _ = srsgpu.make_pusch_demod_configs([to_demod(dict(cfg, **bad))], [0])
        with pytest.raises(srsgpu.SrsGpuError):
            srsgpu.PuschDemodulatorPlan(ctx, arr, 24, 4)


def to_demod_general(cfg, crb=None, tp=False):
    d = to_demod(cfg)
    d.crb_mask, d.transform_precoding = crb, int(tp)
    return d


def check_stats(got, want, nof_layers):
    """Statistics parity: the same rows present (NaN = no data), EVM per symbol 1e-2 relative and total 5e-3, SINR
    5e-3 dB with one layer and 0.1 dB with two (near-singular 2 x 2 REs dominate the mean; see test_golden.py)."""
    assert np.array_equal(np.isnan(got), np.isnan(want)), (got, want)
    ok = ~np.isnan(want)
    np.testing.assert_allclose(got[:14, 1][ok[:14, 1]], want[:14, 1][ok[:14, 1]], rtol=1e-2)
    if ok[14, 1]:
        np.testing.assert_allclose(got[14, 1], want[14, 1], rtol=5e-3)
    np.testing.assert_allclose(got[:, 0][ok[:, 0]], want[:, 0][ok[:, 0]], atol=5e-3 if nof_layers == 1 else 0.1)


def test_pusch_demod_general_golden(ctx):
    """CRB masks, transform precoding and the post-equalization SINR / EVM against the reference's LLRs and statistics
    (tests/golden/pusch_demod_general.npz), every case in ONE plan; executed twice (the plan's accumulators reset)."""
    import srsgpu
    cases = list(G.pusch_demod_general_cases())
    grids, hs, nvs, demods = [], [], [], []
    for cfg, tp, crb, grid, H, nv, _, _ in cases:
        g, h, n = pad_slot(grid, H, nv)
        grids.append(g)
        hs.append(h)
        nvs.append(n)
        demods.append(to_demod_general(cfg, crb, tp))
    dem = srsgpu.PuschDemodulator(ctx, 32, 4)
    for _ in range(2):
        got, stats = dem.demodulate_batch(np.stack(grids), np.stack(hs), np.stack(nvs), demods,
                                          list(range(len(cases))), with_stats=True)
        for i, (cfg, tp, crb, _, _, _, want, wstats) in enumerate(cases):
            ok, st = close(got[i], want)
            assert got[i].size == want.size and ok, (cfg, tp, st)
            check_stats(stats[i], wstats, cfg["nof_layers"])


def test_pusch_demod_general_random_vs_oracle(ctx):
    """48 random transmissions (CRB masks or contiguous, with and without transform precoding, 1..273 PRB) in ONE
    plan over 273-PRB grids, against the restatement (LLRs within one step on < 5 %, statistics as above)."""
    import srsgpu
    from pusch_demod_cases import random_general_case
    rng = np.random.default_rng(77)
    items = []
    for i in range(48):
        tp = i % 3 == 0
        items.append((random_general_case(rng, 273, transform_precoding=tp, mask=i % 2 == 0), tp))
    grids, hs, nvs, demods = [], [], [], []
    for (cfg, grid, H, nv, crb), tp in items:
        g, h, n = pad_slot(grid, H, nv)
        grids.append(g)
        hs.append(h)
        nvs.append(n)
        demods.append(to_demod_general(cfg, crb, tp))
    got, stats = srsgpu.PuschDemodulator(ctx, 273, 4).demodulate_batch(np.stack(grids), np.stack(hs), np.stack(nvs),
                                                                        demods, list(range(len(items))),
                                                                        with_stats=True)
    for i, ((cfg, grid, H, nv, crb), tp) in enumerate(items):
        want, wstats = D.demodulate_ex(cfg, from_bf16(grid), from_bf16(H), nv, crb_mask=crb, transform_precoding=tp)
        ok, st = close(got[i], want)
        assert got[i].size == want.size and ok, (cfg, tp, st)
        check_stats(stats[i], wstats, cfg["nof_layers"])


def test_pusch_demod_general_rejects_invalid(ctx):
    """Transform precoding with two layers or a PRB count that is not 2^a 3^b 5^c, and reserved patterns, fail at plan
    creation (the reference asserts, pusch_demodulator_impl.cpp:347, transform_precoder_dft_impl.cpp)."""
    import srsgpu
    rng = np.random.default_rng(5)
    from pusch_demod_cases import random_case
    cfg, _, _, _ = random_case(rng, 24, nof_layers=2, nof_rx_ports=2)
    cfg.update(rb_start=0, nof_rb=4, dmrs_type2=0, nof_cdm_groups_without_data=2)
    bad = [to_demod_general(cfg, tp=True)]
    cfg1 = dict(cfg, nof_layers=1, nof_rb=7)
    bad.append(to_demod_general(cfg1, tp=True))
    for d in bad:
        arr, _, _ = srsgpu.make_pusch_demod_configs([d], [0])
        with pytest.raises(srsgpu.SrsGpuError):
            srsgpu.PuschDemodulatorPlan(ctx, arr, 24, 4)
    d = to_demod_general(dict(cfg1, nof_rb=8), crb=np.ones(24, np.uint8))
    arr, _, _ = srsgpu.make_pusch_demod_configs([d], [0])
    exts, _keep = srsgpu.make_crb_mask_exts([d], 24)
    exts[0].nof_reserved = 1
    with pytest.raises(srsgpu.SrsGpuError):
        srsgpu.PuschDemodulatorPlan(ctx, arr, 24, 4, exts)
