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


def to_general_mod(cfg, w, crb, grid_prb):
    import srsgpu
    import srsgpu.alloc as A
    m = to_mod(cfg, w)
    m.crb_mask = crb
    m.reserved = [A.ReservedPattern(re_mask=r[1], symbol_mask=r[2], crb_mask=r[0]) for r in cfg["reserved"]]
    m.prg_size = cfg["prg_size"]
    m.prg_weights = cfg["prg_weights"]
    return m


def test_pdsch_modulator_general_golden(ctx):
    """Reference-made grids of general allocations (VRB bitmaps non-interleaved / interleaved, reserved RE patterns,
    single-PRG precoding), one plan with every case, bit-exact."""
    import srsgpu
    cases = list(G.pdsch_mod_general_cases())
    grid_prb = cases[0][2]
    mods = [to_general_mod(c, w, crb, grid_prb) for c, _, _, w, _, _, crb in cases]
    for m, (c, nbits, *_rest) in zip(mods, cases):
        assert m.nof_re(grid_prb) * m.nof_layers * m.modulation_order == nbits
    got = srsgpu.PdschModulator(ctx, grid_prb, 4).modulate_batch([c[4] for c in cases], mods)
    for i, (cfg, nbits, _, w, cw, grid, crb) in enumerate(cases):
        assert np.array_equal(got[i, : cfg["nof_ports"]], grid), (i, cfg)


def test_pdsch_modulator_general_random_vs_oracle(ctx):
    """90 random general allocations in ONE plan (contiguous transmissions mixed in), including multi-PRG precoding
    (PRG sizes 2 and 4) and reserved patterns, against the oracle (PRG of a RE = its CRB / prg_size, the reference's
    mapper test definition; see test_pdsch_modulator_multi_prg_reference_defect)."""
    import srsgpu
    from oracle_lib import pdsch_modulate_general
    from pdsch_mod_cases import crb_mask_test_side, random_general_config
    orc = Oracle()
    rng = np.random.default_rng(22)
    G_ = 52
    mods, cws, want = [], [], []
    for i in range(90):
        if i % 9 == 8:
            cfg, nbits, w = random_config(rng, G_)
            cw = rng.integers(0, 256, (nbits + 7) // 8).astype(np.uint8)
            g = np.zeros((4, 14, 12 * G_, 2), np.uint16)
            orc.pdsch_modulate(cfg, w, cw, nbits, G_, grid=g[: cfg["nof_ports"]])
            mods.append(to_mod(cfg, w))
        else:
            cfg, nbits, w = random_general_config(rng, G_)
            crb = crb_mask_test_side(cfg, G_)
            cw = rng.integers(0, 256, (nbits + 7) // 8).astype(np.uint8)
            g = np.zeros((4, 14, 12 * G_, 2), np.uint16)
            pdsch_modulate_general(orc.lib, cfg, w, cw, nbits, G_, crb_mask=crb, grid=g[: cfg["nof_ports"]])
            mods.append(to_general_mod(cfg, w, crb, G_))
        cws.append(cw)
        want.append(g)
    got = srsgpu.PdschModulator(ctx, G_, 4).modulate_batch(cws, mods)
    for i, (a, b) in enumerate(zip(got, want)):
        assert np.array_equal(a, b), (i, mods[i])


def test_pdsch_modulator_general_full_band(ctx):
    """273 PRB, interleaved (bundle 4) 90 % VRB bitmap, CSI-RS-like and SSB-like reserved patterns, PRG size 4 with
    4 layers of 256QAM: the largest general codeword."""
    import srsgpu
    import srsgpu.alloc as A
    from oracle_lib import pdsch_modulate_general
    orc = Oracle()
    rng = np.random.default_rng(23)
    vrb = (rng.random(273) < 0.9).astype(np.uint8)
    crb = A.vrb_to_crb_mask(vrb, 0, 273, 273, A.interleaved_other(0, 273, 4))
    ssb = np.zeros(273, np.uint8)
    ssb[100:120] = 1
    reserved = [(np.ones(273, np.uint8), 0x111, (1 << 5) | (1 << 12)), (ssb, 0xFFF, 0b111100)]
    cfg = dict(rnti=0x4601, n_id=7, qm=8, nof_layers=4, nof_ports=4, bwp_start_rb=0, bwp_size_rb=273, rb_start=0,
               nof_rb=0, start_symbol=1, nof_symbols=13, dmrs_symbol_mask=(1 << 2) | (1 << 11), dmrs_type2=0,
               nof_cdm_groups_without_data=2, scaling=1.0, vrb_mask=vrb, interleave=4, reserved=reserved, prg_size=4)
    cfg["prg_weights"] = ((rng.normal(size=(69, 4, 4)) + 1j * rng.normal(size=(69, 4, 4))) / 2).astype(np.complex64)
    w = np.eye(4, dtype=np.complex64)
    m = to_general_mod(cfg, w, crb, 273)
    nbits = m.nof_re(273) * 32
    cw = rng.integers(0, 256, nbits // 8).astype(np.uint8)
    want, _ = pdsch_modulate_general(orc.lib, cfg, w, cw, nbits, 273, crb_mask=crb)
    got = srsgpu.PdschModulator(ctx, 273, 4).modulate(cw, m)
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


def to_dmrs(cfg, w, crb_mask=None):
    import srsgpu
    return srsgpu.PdschDmrs(slot_index=cfg["slot"], scrambling_id=cfg["scrambling_id"], n_scid=cfg["n_scid"],
                            dmrs_type=2 if cfg["dmrs_type2"] else 1, nof_layers=cfg["nof_layers"],
                            nof_ports=cfg["nof_ports"], dmrs_symbol_mask=cfg["dmrs_symbol_mask"],
                            reference_point_k_rb=cfg["reference_point_k_rb"], rb_start=cfg["rb_start"],
                            nof_rb=cfg["nof_rb"], amplitude=cfg["amplitude"], weights=w, crb_mask=crb_mask)


def run_dmrs(ctx, items, grid_prb, S, masks=None):
    import torch
    import srsgpu
    dev = torch.device("cuda", 0)
    d_grid = torch.zeros(S * 4 * 14 * 12 * grid_prb, dtype=torch.int32, device=dev)
    masks = masks or [None] * len(items)
    dmrs = [to_dmrs(c, w, m) for (c, w, _), m in zip(items, masks)]
    exts, _keep = srsgpu.make_dmrs_exts(dmrs, grid_prb)
    plan = srsgpu.PdschDmrsPlan(ctx, srsgpu.make_pdsch_dmrs_configs(dmrs, [g for _, _, g in items]), grid_prb, 4,
                                exts)
    plan.execute(d_grid)
    torch.cuda.synchronize()
    plan.close()
    return d_grid.cpu().numpy().view(np.uint16).reshape(S, 4, 14, 12 * grid_prb, 2)


def test_pdsch_dmrs_golden(ctx):
    """PDSCH DM-RS (dmrs_pdsch_processor::map) bit-exact against the reference's grids, all cases in ONE plan."""
    cases = list(G.pdsch_dmrs_cases())
    got = run_dmrs(ctx, [(c, w, i) for i, (c, w, _) in enumerate(cases)], 24, len(cases))
    for i, (cfg, w, want) in enumerate(cases):
        assert np.array_equal(got[i, : cfg["nof_ports"]], want), cfg


def test_pdsch_dmrs_random_vs_oracle(ctx):
    """60 random configurations (1-4 layers / ports, types 1 and 2, double symbols) against the oracle, bit-exact."""
    import pdsch_dmrs_oracle as M
    from pdsch_dmrs_cases import random_config
    rng = np.random.default_rng(31)
    items = [random_config(rng, 52) for _ in range(60)]
    got = run_dmrs(ctx, [(c, w, i) for i, (c, w) in enumerate(items)], 52, len(items))
    for i, (cfg, w) in enumerate(items):
        assert np.array_equal(got[i, : cfg["nof_ports"]], M.dmrs_map(cfg, w, 52)), cfg


def test_pdsch_dmrs_crb_mask_golden(ctx):
    """PDSCH DM-RS over general CRB masks (rb_mask) bit-exact against the reference's grids, in ONE plan together
    with a contiguous transmission."""
    cases = list(G.pdsch_dmrs_mask_cases())
    plain = list(G.pdsch_dmrs_cases())[0]
    items = [(c, w, i) for i, (c, w, _, _) in enumerate(cases)] + [(plain[0], plain[1], len(cases))]
    masks = [m for _, _, m, _ in cases] + [None]
    got = run_dmrs(ctx, items, 51, len(items), masks)
    for i, (cfg, w, _, want) in enumerate(cases):
        assert np.array_equal(got[i, : cfg["nof_ports"]], want), cfg
    import pdsch_dmrs_oracle as M
    assert np.array_equal(got[-1, : plain[0]["nof_ports"]], M.dmrs_map(plain[0], plain[1], 51))


def test_pdsch_dmrs_crb_mask_random_vs_oracle(ctx):
    """40 random CRB-mask configurations against the oracle, bit-exact; reserved patterns / PRGs are rejected."""
    import pdsch_dmrs_oracle as M
    import srsgpu
    from pdsch_dmrs_cases import random_mask_config
    rng = np.random.default_rng(33)
    items = [random_mask_config(rng, 273) for _ in range(40)]
    got = run_dmrs(ctx, [(c, w, i) for i, (c, w, _) in enumerate(items)], 273, len(items), [m for _, _, m in items])
    for i, (cfg, w, m) in enumerate(items):
        assert np.array_equal(got[i, : cfg["nof_ports"]], M.dmrs_map(cfg, w, 273, crb_mask=m)), cfg
    cfg, w, m = items[0]
    d = to_dmrs(cfg, w, m)
    exts, _keep = srsgpu.make_dmrs_exts([d], 273)
    exts[0].prg_size = 4
    with pytest.raises(srsgpu.SrsGpuError):
        srsgpu.PdschDmrsPlan(ctx, srsgpu.make_pdsch_dmrs_configs([d], [0]), 273, 4, exts)
