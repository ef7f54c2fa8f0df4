"""PUSCH demodulator test configurations shared by the oracle-vs-reference tests, the golden-fixture generator and
the GPU parity tests. TEST INFRASTRUCTURE ONLY."""
import numpy as np

import ofdm_oracle
import pusch_demod_oracle as D

QAM_AMP = {2: 1 / np.sqrt(2), 4: 1 / np.sqrt(10), 6: 1 / np.sqrt(42), 8: 1 / np.sqrt(170)}


def bf16(x):
    return ofdm_oracle.complex_to_bf16(x)


def from_bf16(u):
    return ofdm_oracle.bf16_to_complex(u).astype(np.complex64)


def random_case(rng, grid_prb, nof_layers=None, nof_rx_ports=None, qm=None, snr_db=None, max_rb=None):
    """A transmission with random allocation / DM-RS pattern, a random flat-per-RE channel, QAM symbols through it plus
    noise. Returns (cfg, grid (P, 14, nsc, 2) bf16, ch_est (L, P, 14, nsc, 2) bf16, noise_var (P,) float32)."""
    L = int(nof_layers or rng.choice([1, 2]))
    P = int(nof_rx_ports or (rng.choice([1, 2, 3, 4]) if L == 1 else rng.choice([2, 4])))
    q = int(qm or rng.choice([2, 4, 6, 8]))
    nrb = int(rng.integers(1, min(grid_prb, max_rb or grid_prb) + 1))
    rb0 = int(rng.integers(0, grid_prb - nrb + 1))
    start = int(rng.integers(0, 3))
    nsym = int(rng.integers(3, 15 - start))
    mask = 0
    for s in range(start, start + nsym):
        if rng.random() < 0.2:
            mask |= 1 << s
    t2 = int(rng.integers(0, 2))
    cdm = int(rng.integers(1, 4 if t2 else 3))
    cfg = dict(rnti=int(rng.integers(1, 65536)), n_id=int(rng.integers(0, 1024)), qm=q, nof_layers=L, nof_rx_ports=P,
               start_symbol=start, nof_symbols=nsym, dmrs_symbol_mask=mask, dmrs_type2=t2,
               nof_cdm_groups_without_data=cdm, rb_start=rb0, nof_rb=nrb)
    nsc = 12 * grid_prb
    H = (rng.normal(size=(L, P, 14, nsc)) + 1j * rng.normal(size=(L, P, 14, nsc))) / np.sqrt(2)
    snr = float(snr_db if snr_db is not None else rng.uniform(5, 30))
    nv = (10 ** (-snr / 10) * rng.uniform(0.5, 1.5, P)).astype(np.float32)
    lv = np.arange(-(2 ** (q // 2) - 1), 2 ** (q // 2), 2) * QAM_AMP[q]
    x = rng.choice(lv, (L, 14, nsc)) + 1j * rng.choice(lv, (L, 14, nsc))
    Hq = from_bf16(bf16(H))
    y = np.einsum("lpsk,lsk->psk", Hq, x)
    y += (rng.normal(size=y.shape) + 1j * rng.normal(size=y.shape)) * np.sqrt(nv[:, None, None] / 2)
    return cfg, bf16(y), bf16(H), nv


def valid_tp_prbs(limit):
    """PRB counts a transform-precoded allocation may take (TS 38.211 section 6.3.1.4: 2^a 3^b 5^c)."""
    out = []
    for n in range(1, limit + 1):
        m = n
        for f in (2, 3, 5):
            while m % f == 0:
                m //= f
        if m == 1:
            out.append(n)
    return out


def random_general_case(rng, grid_prb, transform_precoding=False, mask=True, nof_rx_ports=None, qm=None,
                        snr_db=None, max_rb=None):
    """random_case with a general CRB mask (RBG runs or scattered CRBs; with transform precoding, a PRB count the DFT
    supports and DM-RS symbols without data). Returns (cfg, grid, ch_est, noise_var, crb_mask or None)."""
    cfg, grid, H, nv = random_case(rng, grid_prb, nof_layers=1 if transform_precoding else None,
                                   nof_rx_ports=nof_rx_ports, qm=qm, snr_db=snr_db, max_rb=max_rb)
    lim = min(grid_prb, max_rb or grid_prb)
    crb = None
    if transform_precoding:
        cfg["dmrs_type2"], cfg["nof_cdm_groups_without_data"] = 0, 2
        nrb = int(rng.choice(valid_tp_prbs(lim)))
    else:
        nrb = int(rng.integers(1, lim + 1))
    if mask:
        crb = np.zeros(grid_prb, np.uint8)
        crb[rng.choice(grid_prb, nrb, replace=False)] = 1
        rbs = np.flatnonzero(crb)
        cfg["rb_start"], cfg["nof_rb"] = int(rbs[0]), nrb
    else:
        cfg["rb_start"], cfg["nof_rb"] = int(rng.integers(0, grid_prb - nrb + 1)), nrb
    return cfg, grid, H, nv, crb

