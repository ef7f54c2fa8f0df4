"""GPU parity of the PDSCH modulator (scrambling, modulation mapping, layer mapping, wideband precoding, RE mapping into
bf16 grids; srsgpu_pdsch_modulator_plan through the C ABI) against the reference's own grids
(tests/golden/pdsch_modulator.npz, made by pdsch_modulator_impl built from its sources) and against the oracle
(oracle/oracle_pdsch.cpp) on random and full-band configurations. Bit-exact: the bf16 grid words must be identical."""
import numpy as np
import pytest

import golden_lib as G
from oracle_lib import Oracle
from pdsch_mod_cases import full_band_config, random_config

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import srsgpu
    return srsgpu.Context(0)


def to_mod(cfg, w):
    import srsgpu
    return srsgpu.PdschModulation(
        rnti=cfg["rnti"], n_id=cfg["n_id"], modulation_order=cfg["qm"], nof_layers=cfg["nof_layers"],
        nof_ports=cfg["nof_ports"], bwp_start_rb=cfg["bwp_start_rb"], bwp_size_rb=cfg["bwp_size_rb"],
        rb_start=cfg["rb_start"], nof_rb=cfg["nof_rb"], start_symbol=cfg["start_symbol"],
        nof_symbols=cfg["nof_symbols"], dmrs_symbol_mask=cfg["dmrs_symbol_mask"], dmrs_type=2 if cfg["dmrs_type2"] else 1,
        nof_cdm_groups_without_data=cfg["nof_cdm_groups_without_data"], scaling=cfg["scaling"], weights=w)


def test_pdsch_modulator_golden(ctx):
    """Every reference-made grid: one transmission per call, grid with the case's ports and PRBs."""
    import srsgpu
    n = 0
    for cfg, nbits, grid_prb, w, cw, grid in G.pdsch_modulator_cases():
        P = cfg["nof_ports"]
        got = srsgpu.PdschModulator(ctx, grid_prb, P).modulate(cw, to_mod(cfg, w))
        assert got.shape == grid.shape
        assert np.array_equal(got, grid), cfg
        n += 1
    assert n > 0


def test_pdsch_modulator_random_batch(ctx):
    """120 random transmissions (QPSK..256QAM, 1-4 layers/ports, DM-RS types 1/2, 1-3 CDM groups, power scalings) in
    ONE plan, each into its own 40-PRB grid, against the oracle."""
    import srsgpu
    orc = Oracle()
    rng = np.random.default_rng(21)
    mods, cws, want = [], [], []
    for _ in range(120):
        cfg, nbits, w = random_config(rng, 40)
        cw = rng.integers(0, 256, (nbits + 7) // 8).astype(np.uint8)
        g = np.zeros((4, 14, 12 * 40, 2), np.uint16)
        orc.pdsch_modulate(cfg, w, cw, nbits, 40, grid=g[: cfg["nof_ports"]])
        mods.append(to_mod(cfg, w))
        cws.append(cw)
        want.append(g)
    got = srsgpu.PdschModulator(ctx, 40, 4).modulate_batch(cws, mods)
    for i, (a, b) in enumerate(zip(got, want)):
        assert np.array_equal(a, b), (i, mods[i])


def test_pdsch_modulator_shared_slot_grid(ctx):
    """A 100 MHz slot shared by 64 UEs (disjoint PRB ranges, 4 layers, 256QAM, one DM-RS symbol) mapped into ONE grid,
    against the oracle applied UE after UE to the same grid."""
    import srsgpu
    orc = Oracle()
    rng = np.random.default_rng(5)
    grid = np.zeros((4, 14, 12 * 273, 2), np.uint16)
    mods, cws = [], []
    rb = 0
    for u in range(64):
        nrb = 5 if u < 17 else 4
        cfg = dict(rnti=0x4601 + u, n_id=int(rng.integers(0, 1024)), qm=8, nof_layers=4, nof_ports=4, bwp_start_rb=0,
                   bwp_size_rb=273, rb_start=rb, nof_rb=nrb, start_symbol=0, nof_symbols=14, dmrs_symbol_mask=1 << 2,
                   dmrs_type2=0, nof_cdm_groups_without_data=2, scaling=1.0)
        rb += nrb
        w = (rng.normal(size=(4, 4)) + 1j * rng.normal(size=(4, 4))).astype(np.complex64) / 2
        m = to_mod(cfg, w)
        nbits = m.nof_re() * 32
        cw = rng.integers(0, 256, nbits // 8).astype(np.uint8)
        orc.pdsch_modulate(cfg, w, cw, nbits, 273, grid=grid)
        mods.append(m)
        cws.append(cw)
    got = srsgpu.PdschModulator(ctx, 273, 4).modulate_batch(cws, mods, grid_index=[0] * 64)
    assert np.array_equal(got[0], grid)


@pytest.mark.parametrize("L,qm", [(1, 2), (2, 4), (3, 6), (4, 8), (4, 2)])
def test_pdsch_modulator_full_band(ctx, L, qm):
    """273 PRB x 14 symbols (the largest codewords: up to 1.36 Mbit, 167 chunks of 8192 bits)."""
    import srsgpu
    orc = Oracle()
    rng = np.random.default_rng(L * 10 + qm)
    cfg, nbits = full_band_config(nof_layers=L, qm=qm)
    w = (rng.normal(size=(4, L)) + 1j * rng.normal(size=(4, L))).astype(np.complex64)
    cw = rng.integers(0, 256, (nbits + 7) // 8).astype(np.uint8)
    want = orc.pdsch_modulate(cfg, w, cw, nbits, 273)
    got = srsgpu.PdschModulator(ctx, 273, 4).modulate(cw, to_mod(cfg, w))
    assert np.array_equal(got, want)


def test_pdsch_modulator_rejects_invalid(ctx):
    """The reference's assertions: time allocation beyond the slot, codeword length not filling the allocation."""
    import srsgpu
    cfg, nbits = full_band_config()
    w = np.eye(4, dtype=np.complex64)
    bad_time = dict(cfg, start_symbol=3, nof_symbols=12)
    with pytest.raises(srsgpu.SrsGpuError):
        arr = srsgpu.make_pdsch_mod_configs([to_mod(bad_time, w)], [0], [0])
        srsgpu.PdschModulatorPlan(ctx, arr, 273, 4)
    arr = srsgpu.make_pdsch_mod_configs([to_mod(cfg, w)], [0], [0])
    arr[0].nof_bits -= 32
    with pytest.raises(srsgpu.SrsGpuError):
        srsgpu.PdschModulatorPlan(ctx, arr, 273, 4)
