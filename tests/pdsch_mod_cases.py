"""PDSCH modulator test configurations shared by the oracle-vs-reference tests, the golden-fixture generator
(tools/gen_golden.py) and the GPU parity tests. TEST INFRASTRUCTURE ONLY."""
import numpy as np

from oracle_lib import pdsch_mod_nof_re


def random_config(rng, grid_nof_prb, max_rb=None, qm=None, nof_layers=None, nof_ports=None):
    """A random valid configuration: contiguous VRB allocation inside a BWP, random symbols and DM-RS symbols (type 1
    or 2, 1..3 CDM groups without data) and at most 156 data REs per PRB (the reference's per-codeword buffer bound,
    pdsch_constants.h:63). Returns (cfg, nof_bits, weights (ports x layers complex64))."""
    while True:
        L = int(nof_layers or rng.integers(1, 5))
        P = int(nof_ports or rng.integers(L, 5))
        q = int(qm or rng.choice([2, 4, 6, 8]))
        bwp_start = int(rng.integers(0, min(4, grid_nof_prb)))
        bwp_size = grid_nof_prb - bwp_start
        nof_rb = int(rng.integers(1, min(bwp_size, max_rb or bwp_size) + 1))
        rb_start = int(rng.integers(0, bwp_size - nof_rb + 1))
        start = int(rng.integers(0, 4))
        nsym = int(rng.integers(1, 15 - start))
        mask = 0
        for sym in range(start, start + nsym):
            if rng.random() < 0.25:
                mask |= 1 << sym
        t2 = int(rng.integers(0, 2))
        cdm = int(rng.integers(1, 4 if t2 else 3))
        cfg = dict(rnti=int(rng.integers(1, 65536)), n_id=int(rng.integers(0, 1024)), qm=q, nof_layers=L, nof_ports=P,
                   bwp_start_rb=bwp_start, bwp_size_rb=bwp_size, rb_start=rb_start, nof_rb=nof_rb,
                   start_symbol=start, nof_symbols=nsym, dmrs_symbol_mask=mask, dmrs_type2=t2,
                   nof_cdm_groups_without_data=cdm, scaling=float(rng.choice([1.0, 0.7071, 0.0, 2.5, 0.31])))
        nre = pdsch_mod_nof_re(cfg)
        if nre == 0 or nre > 156 * nof_rb:
            continue
        w = (rng.normal(size=(P, L)) + 1j * rng.normal(size=(P, L))).astype(np.complex64)
        return cfg, nre * L * q, w


def full_band_config(nof_layers=4, qm=8, rnti=0x4601, n_id=500):
    """100 MHz (273 PRB) allocation, 14 symbols, one DM-RS symbol (type 1, 2 CDM groups: no data in it)."""
    cfg = dict(rnti=rnti, n_id=n_id, qm=qm, nof_layers=nof_layers, nof_ports=4, bwp_start_rb=0, bwp_size_rb=273,
               rb_start=0, nof_rb=273, start_symbol=0, nof_symbols=14, dmrs_symbol_mask=1 << 2, dmrs_type2=0,
               nof_cdm_groups_without_data=2, scaling=1.0)
    return cfg, pdsch_mod_nof_re(cfg) * nof_layers * qm
