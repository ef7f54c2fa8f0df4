"""PUSCH channel-estimation test cases shared by the oracle-vs-reference tests, the golden-fixture generator and the
GPU parity tests: a received slot grid with DM-RS (port 1000) through a frequency-selective channel plus noise.
TEST INFRASTRUCTURE ONLY."""
import numpy as np

import pusch_chest_oracle as C
from pusch_demod_cases import bf16


def random_crb_mask(rng, grid_prb, nof_rb=None):
    """A non-contiguous CRB mask: RBG-like runs or scattered CRBs (at least two runs)."""
    while True:
        if rng.random() < 0.5:
            rbg = int(rng.choice([2, 4, 8]))
            sel = rng.random((grid_prb + rbg - 1) // rbg) < rng.uniform(0.2, 0.8)
            m = np.repeat(sel, rbg)[:grid_prb].astype(np.uint8)
        else:
            m = (rng.random(grid_prb) < rng.uniform(0.1, 0.8)).astype(np.uint8)
        if nof_rb is not None and m.sum() > nof_rb:
            m[np.flatnonzero(m)[nof_rb:]] = 0
        rbs = np.flatnonzero(m)
        if rbs.size >= 2 and rbs[-1] - rbs[0] + 1 != rbs.size:
            return m


def random_case(rng, grid_prb, nof_rx_ports=None, nof_rb=None, dmrs_type2=None, snr_db=None, dmrs_mask=None,
                cfo_hz=0.0, delay=0.0, numerology=1, crb_mask=None, low_papr_id=None):
    """Returns (cfg, grid (P, 14, nsc, 2) bf16, true channel (P, nsc) complex). cfo_hz rotates OFDM symbol l by
    2 pi cfo t_l (t_l: the symbol's start epoch); delay (in samples of a 4096-point DFT, may be negative) shifts every
    path. crb_mask: the DM-RS go to those CRBs (cfg rb_start / nof_rb = its first CRB / CRB count). low_papr_id: the
    DM-RS is the low-PAPR sequence of group low_papr_id mod 30 (transform precoding, type 1)."""
    P = int(nof_rx_ports or rng.integers(1, 5))
    nrb = int(nof_rb or rng.integers(1, grid_prb + 1))
    rb0 = int(rng.integers(0, grid_prb - nrb + 1))
    rbs = list(range(rb0, rb0 + nrb))
    if crb_mask is not None:
        rbs = [int(i) for i in np.flatnonzero(crb_mask)]
        rb0, nrb = rbs[0], len(rbs)
    t2 = int(dmrs_type2 if dmrs_type2 is not None else rng.integers(0, 2))
    start = int(rng.integers(0, 2))
    nsym = int(rng.integers(6, 15 - start))
    if dmrs_mask is None:
        cand = [l for l in range(start, start + nsym)]
        k = int(rng.integers(1, 4))
        dmrs_mask = sum(1 << l for l in sorted(rng.choice(cand, k, replace=False)))
    cfg = dict(slot=int(rng.integers(0, 20)), scrambling_id=int(rng.integers(0, 65536)), n_scid=int(rng.integers(0, 2)),
               dmrs_type2=t2, scaling=float(rng.choice([1.0, 1.4125375, 0.7071])), dmrs_symbol_mask=int(dmrs_mask),
               start_symbol=start, nof_symbols=nsym, rb_start=rb0, nof_rb=nrb, nof_rx_ports=P)
    nsc = 12 * grid_prb
    k = np.arange(nsc)
    H = np.zeros((P, nsc), np.complex128)
    for p in range(P):
        for _ in range(4):
            tau = rng.uniform(0, 40)
            H[p] += (rng.normal() + 1j * rng.normal()) / np.sqrt(8) * np.exp(-2j * np.pi * k * (tau + delay) / 4096)
    snr = float(snr_db if snr_db is not None else rng.uniform(5, 35))
    nv = 10 ** (-snr / 10)
    x = (rng.choice([-1, 1], (14, nsc)) + 1j * rng.choice([-1, 1], (14, nsc))) / np.sqrt(2)
    pat = C.layer0_pattern(t2)
    sc = np.array([rb * 12 + q for rb in rbs for q in pat])
    for l in range(14):
        if (dmrs_mask >> l) & 1:
            if low_papr_id is not None:
                x[l, sc] = cfg["scaling"] * C.low_papr_sequence(low_papr_id % 30, sc.size)
            else:
                x[l, sc] = cfg["scaling"] * C.dmrs_sequence(cfg["slot"], l, cfg["scrambling_id"], cfg["n_scid"], t2,
                                                            rb0, nrb, rbs)
    y = H[:, None, :] * x[None]
    if cfo_hz:
        ep = C.symbol_start_epochs(numerology)
        y = y * np.exp(2j * np.pi * cfo_hz / ((15 << numerology) * 1000.0) * ep)[None, :, None]
    y = y + (rng.normal(size=(P, 14, nsc)) + 1j * rng.normal(size=(P, 14, nsc))) * np.sqrt(nv / 2)
    return cfg, bf16(y), H


def multilayer_case(rng, grid_prb, nof_layers, nof_rx_ports, nof_rb, rb_start=0, snr_db=30.0, dmrs_mask=(1 << 2)):
    """Layers 0..L-1 on DM-RS ports 1000..1003 (type 1, CDM groups 0/1, w_f = (+1, -1) for ports 1001 / 1003) through
    a smooth random channel per (port, layer). Returns (cfg, grid bf16, true channel (L, P, nsc))."""
    P, L = nof_rx_ports, nof_layers
    cfg = dict(slot=int(rng.integers(0, 20)), scrambling_id=int(rng.integers(0, 65536)), n_scid=0, dmrs_type2=0,
               scaling=1.4125375, dmrs_symbol_mask=int(dmrs_mask), start_symbol=0, nof_symbols=14, rb_start=rb_start,
               nof_rb=nof_rb, nof_rx_ports=P, nof_layers=L)
    nsc = 12 * grid_prb
    k = np.arange(nsc)
    H = np.zeros((L, P, nsc), np.complex128)
    for ly in range(L):
        for p in range(P):
            for _ in range(3):
                tau = rng.uniform(0, 12)
                H[ly, p] += (rng.normal() + 1j * rng.normal()) / np.sqrt(6) * np.exp(-2j * np.pi * k * tau / 4096)
    nv = 10 ** (-snr_db / 10)
    x = (rng.choice([-1, 1], (L, 14, nsc)) + 1j * rng.choice([-1, 1], (L, 14, nsc))) / np.sqrt(2) / np.sqrt(L)
    for l in range(14):
        if (dmrs_mask >> l) & 1:
            x[:, l, :] = 0
            seq = C.dmrs_sequence(cfg["slot"], l, cfg["scrambling_id"], 0, 0, rb_start, nof_rb)
            for ly in range(L):
                g = ly // 2
                sc = np.array([(rb_start + rb) * 12 + g + 2 * j for rb in range(nof_rb) for j in range(6)])
                wf = np.where(np.arange(sc.size) % 2 == 1, -1.0 if ly % 2 else 1.0, 1.0)
                x[ly, l, sc] = cfg["scaling"] * seq * wf
    y = np.einsum("lpk,lsk->psk", H, x)
    y += (rng.normal(size=y.shape) + 1j * rng.normal(size=y.shape)) * np.sqrt(nv / 2)
    return cfg, bf16(y), H
