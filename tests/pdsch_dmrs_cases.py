"""PDSCH DM-RS test configurations (oracle-vs-reference tests, golden generator, GPU tests). TEST INFRASTRUCTURE
ONLY."""
import numpy as np


def random_config(rng, grid_prb, nof_layers=None, nof_ports=None):
    L = int(nof_layers or rng.integers(1, 5))
    P = int(nof_ports or rng.integers(L, 5))
    nrb = int(rng.integers(1, grid_prb + 1))
    rb0 = int(rng.integers(0, grid_prb - nrb + 1))
    mask = 0
    for l in sorted(rng.choice(np.arange(1, 14), int(rng.integers(1, 4)), replace=False)):
        mask |= 1 << int(l)
        if rng.random() < 0.3 and l + 1 < 14:  # double-symbol DM-RS
            mask |= 1 << int(l + 1)
    cfg = dict(slot=int(rng.integers(0, 20)), scrambling_id=int(rng.integers(0, 65536)), n_scid=int(rng.integers(0, 2)),
               dmrs_type2=int(rng.integers(0, 2)), nof_layers=L, nof_ports=P, dmrs_symbol_mask=mask,
               reference_point_k_rb=int(rng.integers(0, rb0 + 1)), rb_start=rb0, nof_rb=nrb,
               amplitude=float(rng.choice([1.0, 1.4125375, 0.5])))
    w = ((rng.normal(size=(P, L)) + 1j * rng.normal(size=(P, L))) / 2).astype(np.complex64)
    return cfg, w


def random_mask_config(rng, grid_prb, nof_layers=None, nof_ports=None):
    """A random configuration with a general CRB mask (rb_mask): type-0 style RBG runs or a random scatter, the
    sequence reference point at or below the first allocated CRB. Returns (cfg, weights, crb_mask)."""
    cfg, w = random_config(rng, grid_prb, nof_layers, nof_ports)
    if rng.random() < 0.5:
        rbg = int(rng.choice([2, 4, 8, 16]))
        sel = rng.random((grid_prb + rbg - 1) // rbg) < rng.uniform(0.2, 0.8)
        mask = np.repeat(sel, rbg)[:grid_prb].astype(np.uint8)
    else:
        mask = (rng.random(grid_prb) < rng.uniform(0.1, 0.9)).astype(np.uint8)
    if not mask.any():
        mask[int(rng.integers(0, grid_prb))] = 1
    first = int(np.flatnonzero(mask)[0])
    cfg.update(rb_start=first, nof_rb=int(mask.sum()), reference_point_k_rb=int(rng.integers(0, first + 1)))
    return cfg, w, mask
