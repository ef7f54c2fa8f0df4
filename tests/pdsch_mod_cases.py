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


def general_nof_re(cfg, crb_mask, grid_nof_prb):
    """Data REs of a general allocation (test-side count, independent of the product's srsgpu.alloc): allocated CRBs x
    symbols minus the BWP DM-RS pattern on DM-RS symbols and the reserved patterns."""
    if cfg["dmrs_type2"]:
        dm = {k for k in range(12) if (k % 6) // 2 < cfg["nof_cdm_groups_without_data"]}
    else:
        dm = {k for k in range(12) if k % 2 < cfg["nof_cdm_groups_without_data"]}
    n = 0
    b0, b1 = cfg["bwp_start_rb"], cfg["bwp_start_rb"] + cfg["bwp_size_rb"]
    for l in range(cfg["start_symbol"], cfg["start_symbol"] + cfg["nof_symbols"]):
        for crb in range(grid_nof_prb):
            if not crb_mask[crb]:
                continue
            excl = set(dm) if ((cfg["dmrs_symbol_mask"] >> l) & 1 and b0 <= crb < b1) else set()
            for rc, rre, rsym in cfg["reserved"]:
                if (rsym >> l) & 1 and rc[crb]:
                    excl |= {k for k in range(12) if (rre >> k) & 1}
            n += 12 - len(excl)
    return n


def random_general_config(rng, grid_nof_prb, interleave=None, prg=None, nof_reserved=None):
    """A random general allocation: random type-0 VRB bitmap of the BWP mapped non-interleaved or interleaved (bundle
    size 2 / 4, vrb_to_prb::create_interleaved_other), 0..3 reserved RE patterns (random CRB subsets, PRB subcarriers and
    symbols, e.g. CSI-RS / SSB-like), wideband or per-PRG precoding (PRG sizes 2 / 4 / whole grid). Returns (cfg with
    vrb_mask, interleave, reserved [(crb mask, re mask, symbol mask)], prg_size, prg_weights; nof_bits; weights)."""
    while True:
        cfg, _, w = random_config(rng, grid_nof_prb)
        bwp_start = int(rng.integers(0, min(6, grid_nof_prb - 8)))
        bwp_size = int(rng.integers(8, grid_nof_prb - bwp_start + 1))
        cfg.update(bwp_start_rb=bwp_start, bwp_size_rb=bwp_size, rb_start=0, nof_rb=0)
        il = int(rng.choice([0, 0, 2, 4]) if interleave is None else interleave)
        nvrb = bwp_size
        density = float(rng.choice([0.2, 0.5, 0.9, 1.0]))
        vrb = (rng.random(nvrb) < density).astype(np.uint8)
        if not vrb.any():
            vrb[int(rng.integers(0, nvrb))] = 1
        reserved = []
        for _ in range(int(rng.integers(0, 4) if nof_reserved is None else nof_reserved)):
            rc = (rng.random(grid_nof_prb) < rng.choice([0.3, 1.0])).astype(np.uint8)
            if not rc.any():
                rc[int(rng.integers(0, grid_nof_prb))] = 1
            rre = int(rng.integers(1, 4096))
            rsym = int(rng.integers(1, 1 << 14))
            reserved.append((rc, rre, rsym))
        P, L = cfg["nof_ports"], cfg["nof_layers"]
        prg_size = int(rng.choice([0, 2, 4, grid_nof_prb]) if prg is None else prg)
        nof_prg = -(-grid_nof_prb // prg_size) if prg_size else 0
        prg_w = ((rng.normal(size=(nof_prg, P, L)) + 1j * rng.normal(size=(nof_prg, P, L))).astype(np.complex64)
                 if prg_size else None)
        cfg.update(vrb_mask=vrb, interleave=il, reserved=reserved, prg_size=prg_size, prg_weights=prg_w)
        crbs = crb_mask_test_side(cfg, grid_nof_prb)
        nre = general_nof_re(cfg, crbs, grid_nof_prb)
        if nre == 0 or nre > 156 * int(crbs.sum()):
            continue
        return cfg, nre * L * cfg["qm"], w


def crb_mask_test_side(cfg, grid_nof_prb):
    """CRB mask of a case, restated on the test side from TS 38.211 7.3.1.6 (vrb_to_prb.cpp:94 interleaver), so the
    product's srsgpu.alloc.vrb_to_crb_mask is checked against the reference's get_crb_mask and not against itself."""
    s, n, L = cfg["bwp_start_rb"], cfg["bwp_size_rb"], cfg["interleave"]
    vrbs = np.flatnonzero(cfg["vrb_mask"])
    if L:
        nb = -(-(n + s % L) // L)
        first = L - s % L
        last = (s + n) % L or L
        prb = list(range(first))
        mid = [None] * (nb - 2)
        C = nb // 2
        for c in range(C):
            for r in range(2):
                j = c * 2 + r
                if j == 0 or j > nb - 2:
                    continue
                mid[j - 1] = r * C + c
        for fj in mid:
            prb += [(fj - 1) * L + first + i for i in range(L)]
        prb += [(nb - 2) * L + first + i for i in range(last)]
        prbs = np.array(prb)[vrbs]
    else:
        prbs = vrbs
    out = np.zeros(grid_nof_prb, np.uint8)
    out[s + prbs] = 1
    return out
