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
