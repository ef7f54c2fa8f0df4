"""273-PRB uplink slots like the test-mode UL (configs[4]: one 273-PRB UE, 256QAM, DM-RS symbols 2 + 11, four rx ports,
CFO compensation) as received grids, shared by the reference-build variance test (CPU) and the GPU LLR parity test.
TEST INFRASTRUCTURE ONLY."""
import numpy as np

import pusch_chest_oracle as C
from pusch_demod_cases import bf16

DMRS_BETA = 10 ** (3 / 20)  # two CDM groups without data (TS 38.214 6.2.2), as srsgpu/slot.py
DMRS_MASK = (1 << 2) | (1 << 11)
NOF_PRB = 273
P = 4


def qam256(rng, n):
    """Random 256QAM points with unit average power (TS 38.211 5.1.5 amplitudes)."""
    lv = np.arange(-15, 16, 2)
    return (rng.choice(lv, n) + 1j * rng.choice(lv, n)) / np.sqrt(170.0)


def ul273_case(rng, snr_db=26.0, cfo_hz_max=300.0, slot=7):
    """Returns (chest cfg, demod cfg, grid (P, 14, nsc, 2) bf16): DM-RS (port 1000, type 1) and 256QAM data through a
    4-path channel per rx port with a random CFO, plus AWGN at snr_db (per RE, unit data power)."""
    nsc = 12 * NOF_PRB
    cfg = dict(slot=slot, scrambling_id=500, n_scid=0, dmrs_type2=0, scaling=DMRS_BETA, dmrs_symbol_mask=DMRS_MASK,
               start_symbol=0, nof_symbols=14, rb_start=0, nof_rb=NOF_PRB, nof_rx_ports=P)
    dcfg = dict(rnti=0x4601, n_id=500, qm=8, nof_layers=1, nof_rx_ports=P, start_symbol=0, nof_symbols=14,
                dmrs_symbol_mask=DMRS_MASK, dmrs_type2=0, nof_cdm_groups_without_data=2, rb_start=0, nof_rb=NOF_PRB)
    k = np.arange(nsc)
    H = np.zeros((P, nsc), np.complex128)
    for p in range(P):
        for _ in range(4):
            tau = rng.uniform(0, 40)
            H[p] += (rng.normal() + 1j * rng.normal()) / np.sqrt(8) * np.exp(-2j * np.pi * k * tau / 4096)
    x = np.zeros((14, nsc), np.complex128)
    rbs = list(range(NOF_PRB))
    sc = np.array([rb * 12 + q for rb in rbs for q in C.layer0_pattern(0)])
    for l in range(14):
        if (DMRS_MASK >> l) & 1:
            x[l, sc] = DMRS_BETA * C.dmrs_sequence(slot, l, 500, 0, 0, 0, NOF_PRB, rbs)
        else:
            x[l] = qam256(rng, nsc)
    y = H[:, None, :] * x[None]
    cfo = rng.uniform(-cfo_hz_max, cfo_hz_max)
    y = y * np.exp(2j * np.pi * cfo / 30000.0 * C.symbol_start_epochs(1))[None, :, None]
    nv = 10 ** (-snr_db / 10)
    y = y + (rng.normal(size=y.shape) + 1j * rng.normal(size=y.shape)) * np.sqrt(nv / 2)
    return cfg, dcfg, bf16(y)


def llr_stats(a, b):
    d = np.abs(a.astype(np.int16) - b.astype(np.int16))
    return dict(n=int(d.size), equal=float(np.mean(d == 0)), within1=float(np.mean(d <= 1)), max=int(d.max()),
                over1=int(np.sum(d > 1)))
