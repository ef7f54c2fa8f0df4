"""TEST INFRASTRUCTURE ONLY — numpy restatement ("oracle") of the srsRAN PUSCH DM-RS channel estimator for one
single-layer transmission (the open-source reference supports one layer: port_channel_estimator_average_impl.cpp:83
asserts it), in float64. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, as the
checker.

Pinned against the reference's own dmrs_pusch_estimator_impl + port_channel_estimator_average_impl (linear
interpolator, DFT time-alignment estimator) built from its sources (oracle/ref/ref_pusch_chest.cpp in
oracle/_ref/libsrsref.so) by tests/test_oracle_vs_reference.py and tests/golden/pusch_chest.npz. The reference computes
in float32 (AVX2), the restatement in float64: estimates and noise variances agree within a stated tolerance.

Reference files (under /root/reference/lib/phy/):
  upper/signal_processors/dmrs_pusch_estimator_impl.cpp:69   DM-RS sequence: c_init = ((14 n_slot + l + 1)
                                                             (2 N_ID + 1) 2^17 + 2 N_ID + n_SCID) mod 2^31, QPSK
                                                             amplitude 1/sqrt(2), sequence index from point A (:98)
  upper/signal_processors/dmrs_helper.cpp:36                 layer RE patterns and w_f / w_t cover codes
  upper/signal_processors/port_channel_estimator_helpers.cpp:143  pilots extracted at the layer pattern of the
                                                             allocated RBs, ascending subcarrier
  upper/signal_processors/port_channel_estimator_average_impl.cpp:154  LSE rx conj(p) summed over the DM-RS symbols
                                                             ("average"), scaled by 1 / (beta D), FD smoothing,
                                                             RSRP / EPRE / noise, frequency interpolation, the same
                                                             estimate for every symbol of the allocation
  upper/signal_processors/port_channel_estimator_helpers.cpp:203  "filter" smoothing: raised-cosine FIR (roll-off 0.2,
                                                             3-symbol span, 10 samples per symbol) resampled to the
                                                             pilot stride over min(nof_rb, 3) RBs, renormalised; virtual
                                                             pilots by linear regression of |p| and the unwrapped arg
                                                             (:307); "same" convolution
  support/interpolator/interpolator_linear_impl.cpp:29      linear between pilots (offset, stride of the pattern),
                                                             first / last pilot held outside
  upper/signal_processors/port_channel_estimator_average_impl.cpp:422  noise: sum |rx - beta f p|^2 / (N D - 1),
                                                             bounded below by RSRP / 10^(100/10)
"""
import numpy as np

import pusch_demod_oracle as D

MAX_V_PILOTS = 12


def rc_filter_taps():
    """31-tap raised cosine (roll-off 0.2) at 10 samples per symbol, n = -15..15 (any global scale: the estimator
    renormalises the taps it uses)."""
    t = np.arange(-15, 16) / 10.0
    beta = 0.2
    with np.errstate(divide="ignore", invalid="ignore"):
        h = np.sinc(t) * np.cos(np.pi * beta * t) / (1 - (2 * beta * t) ** 2)
    sing = np.isclose(np.abs(2 * beta * t), 1.0)
    h[sing] = np.pi / 4 * np.sinc(1 / (2 * beta))
    return h


def layer0_pattern(dmrs_type2):
    """RE pattern of DM-RS port 1000 within a PRB (dmrs_helper.cpp RE_PATTERN_TYPE1_DELTA0 / TYPE2_DELTA0)."""
    return [0, 1, 6, 7] if dmrs_type2 else [0, 2, 4, 6, 8, 10]


def dmrs_sequence(slot, symbol, scrambling_id, n_scid, dmrs_type2, rb_start, nof_rb):
    """DM-RS symbols of the allocated RBs of one OFDM symbol (QPSK, amplitude 1/sqrt(2))."""
    c_init = ((14 * slot + symbol + 1) * (2 * scrambling_id + 1) * (1 << 17) + 2 * scrambling_id + n_scid) % (1 << 31)
    per_rb = 4 if dmrs_type2 else 6
    m0 = rb_start * per_rb
    n = nof_rb * per_rb
    c = D.gold_sequence(c_init, 2 * (m0 + n)).astype(np.float64)
    a = 1 / np.sqrt(2)
    return ((1 - 2 * c[2 * m0::2]) * a + 1j * (1 - 2 * c[2 * m0 + 1::2]) * a)[:n]


def virtual_pilots(base, is_start):
    """compute_v_pilots: linear regression of |p| and unwrap(arg p) over x = 0..n-1, evaluated at x = -n..-1 (start)
    or n..2n-1 (end)."""
    n = base.size
    x = np.arange(n, dtype=np.float64)
    ab = np.abs(base)
    ar = np.unwrap(np.angle(base))
    mean_x = (n - 1) / 2.0
    norm_x_sq = (n - 1) * n * (2 * n - 1) / 6.0
    den = norm_x_sq - n * mean_x * mean_x
    s_abs = (np.dot(ab, x) - mean_x * ab.mean() * n) / den
    i_abs = ab.mean() - s_abs * mean_x
    s_arg = (np.dot(ar, x) - mean_x * ar.mean() * n) / den
    i_arg = ar.mean() - s_arg * mean_x
    xv = np.arange(n) + (-n if is_start else n)
    rho = s_abs * xv + i_abs
    return np.abs(rho) * np.exp(1j * (s_arg * xv + i_arg + np.where(rho > 0, 0.0, np.pi)))


def fd_smoothing(pilots, nof_rb, stride, strategy):
    if strategy == "none":
        return pilots.copy()
    if strategy == "mean":
        return np.full_like(pilots, pilots.mean())
    rc = rc_filter_taps()
    nrb = min(nof_rb, 3)
    half = (nrb * 10 + 1) // 2 // stride
    first = 15 - half * stride
    taps = rc[first: first + (2 * half) * stride + 1: stride]
    taps = taps / taps.sum()
    nv = min(MAX_V_PILOTS, taps.size // 2)
    if nof_rb == 1:
        nv = pilots.size
    enlarged = np.concatenate([virtual_pilots(pilots[:nv], True), pilots, virtual_pilots(pilots[-nv:], False)])
    return np.convolve(enlarged, taps, mode="same")[nv: nv + pilots.size]


def interpolate(pilots, offset, stride, nof_re):
    """interpolator_linear_impl: pilots at offset + i stride, linear in between, the first / last pilot held."""
    out = np.empty(nof_re, np.complex128)
    pos = offset + stride * np.arange(pilots.size)
    out[: offset + 1] = pilots[0]
    for i in range(pilots.size - 1):
        for j in range(1, stride + 1):
            if pos[i] + j < nof_re:
                out[pos[i] + j] = pilots[i] + (pilots[i + 1] - pilots[i]) * j / stride
    last = min(pos[-1], nof_re - 1)
    out[last:] = pilots[-1]
    return out


def estimate(cfg, grid, fd="filter"):
    """cfg: slot, scrambling_id, n_scid, dmrs_type2, scaling (beta), dmrs_symbol_mask, start_symbol, nof_symbols,
    rb_start, nof_rb, nof_rx_ports. grid (P, 14, nsc) complex. Returns (ch (P, 14, nsc) complex128 filled on the
    allocation, noise_var (P,), rsrp (P,), epre (P,), CFO phase between the first two DM-RS symbols (P,) or None when
    there is one DM-RS symbol)."""
    P = cfg["nof_rx_ports"]
    t2 = cfg["dmrs_type2"]
    beta = cfg["scaling"]
    pat = layer0_pattern(t2)
    offset, stride = pat[0], pat[1] - pat[0]
    rb0, nrb = cfg["rb_start"], cfg["nof_rb"]
    sc = np.array([(rb0 + rb) * 12 + k for rb in range(nrb) for k in pat])
    syms = [l for l in range(cfg["start_symbol"], cfg["start_symbol"] + cfg["nof_symbols"])
            if (cfg["dmrs_symbol_mask"] >> l) & 1]
    Dn = len(syms)
    N = sc.size
    pil = [dmrs_sequence(cfg["slot"], l, cfg["scrambling_id"], cfg["n_scid"], t2, rb0, nrb) for l in syms]
    nsc = grid.shape[2]
    ch = np.zeros((P, 14, nsc), np.complex128)
    nvar, rsrp, epre, cfo = np.zeros(P), np.zeros(P), np.zeros(P), [None] * P
    for p in range(P):
        rx = [grid[p, l, sc].astype(np.complex128) for l in syms]
        lse = [r * np.conj(q) for r, q in zip(rx, pil)]
        if Dn > 1:  # CFO phase between the first two DM-RS symbols: arg(sum lse_1 conj(lse_0)) (:350)
            cfo[p] = float(np.angle(np.dot(np.conj(lse[0]), lse[1])))
        f = sum(lse) / (beta * Dn)
        f = fd_smoothing(f, nrb, stride, fd)
        epre[p] = sum(np.sum(np.abs(r) ** 2) for r in rx) / (N * Dn)
        rsrp[p] = np.sum(np.abs(f) ** 2) * beta * beta * Dn / (N * Dn)
        noise = sum(np.sum(np.abs(r - f * beta * q) ** 2) for r, q in zip(rx, pil))
        nvar[p] = max(rsrp[p] / 1e10, noise / (N * Dn - 1))
        fr = interpolate(f, offset, stride, nrb * 12)
        for l in range(cfg["start_symbol"], cfg["start_symbol"] + cfg["nof_symbols"]):
            ch[p, l, rb0 * 12: (rb0 + nrb) * 12] = fr
    return ch, nvar, rsrp, epre, cfo
