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


def dmrs_sequence(slot, symbol, scrambling_id, n_scid, dmrs_type2, rb_start, nof_rb, rbs=None):
    """DM-RS symbols of the allocated RBs of one OFDM symbol (QPSK, amplitude 1/sqrt(2)): the contiguous
    [rb_start, rb_start + nof_rb), or the CRB list `rbs` (dmrs_sequence_generate skips the unallocated CRBs,
    dmrs_helper.cpp:64; reference point A, dmrs_pusch_estimator_impl.cpp:103)."""
    c_init = ((14 * slot + symbol + 1) * (2 * scrambling_id + 1) * (1 << 17) + 2 * scrambling_id + n_scid) % (1 << 31)
    per_rb = 4 if dmrs_type2 else 6
    rbs = list(range(rb_start, rb_start + nof_rb)) if rbs is None else list(rbs)
    m = np.array([rb * per_rb + j for rb in rbs for j in range(per_rb)])
    c = D.gold_sequence(c_init, 2 * (int(m.max()) + 1)).astype(np.float64)
    a = 1 / np.sqrt(2)
    return (1 - 2 * c[2 * m]) * a + 1j * (1 - 2 * c[2 * m + 1]) * a


def _largest_prime_below(n):
    for p in range(n - 1, 1, -1):
        if all(p % d for d in range(2, int(p ** 0.5) + 1)):
            return p
    raise ValueError(n)


def low_papr_sequence(u, m, v=0):
    """TS 38.211 section 5.2.2 low-PAPR base sequence r_(u,v)(n), alpha = 0, as low_papr_sequence_generator_impl.cpp
    builds it (phase tables for M_ZC = 6..24, the length-30 formula, Zadoff-Chu with the largest prime N_ZC < M_ZC and
    q from the float q_hat = N_ZC (u + 1) / 31 above): exp(j pi arg(n) / N_ZC)."""
    import low_papr_tables
    if m in low_papr_tables.PHI:
        return np.exp(1j * np.pi * np.array(low_papr_tables.PHI[m][u]) / 4)
    if m == 30:
        n = np.arange(30)
        return np.exp(1j * np.pi * -(((u + 1) * (n + 1) * (n + 2)) % 62) / 31)
    if m < 36:
        raise ValueError(m)
    nzc = _largest_prime_below(m)
    q_hat = np.float32(np.float32(nzc) * np.float32(u + 1)) / np.float32(31)
    q = int(np.float32(float(q_hat) + 0.5 + v)) if int(np.float32(2) * q_hat) % 2 == 0 \
        else int(np.float32(float(q_hat) + 0.5 - v))
    mm = np.arange(m) % nzc
    return np.exp(1j * np.pi * -((q * mm * (mm + 1)) % (2 * nzc)) / nzc)


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


def symbol_start_epochs(numerology):
    """initialize_symbol_start_epochs (port_channel_estimator_average_impl.cpp:496): cumulative CP durations in units of
    the symbol duration plus the symbol index, normal CP; the +16 kappa CP of cyclic_prefix::get_length
    (cyclic_prefix.h:93) applies to symbols 0 and 7 * 2^mu of the slot."""
    t_c = 1.0 / (480000 * 4096)
    scs_hz = (15 << numerology) * 1000
    ep = np.zeros(14)
    for i in range(14):
        kappa = (144 >> numerology) + (16 if i in (0, 7 << numerology) else 0)
        d = kappa * 64 * t_c * scs_hz
        ep[i] = d if i == 0 else ep[i - 1] + d + 1.0
    return ep


TA_MAX_NOF_RE = 275 * 12   # time_alignment_estimator_dft_impl.h:41 (MAX_NOF_PRBS * NRE)
TA_MAX_DFT = 4096          # pow2(log2_ceil(3300))
TA_MIN_DFT = 128           # 1 / (15 kHz x one 15 kHz TA step), time_alignment_estimator_dft_impl.cpp:96


def ta_dft_size(nof_re):
    """get_idft (time_alignment_estimator_dft_impl.cpp:216): guard-scaled, next power of two, at least 128."""
    n = nof_re * TA_MAX_DFT // TA_MAX_NOF_RE
    size = 1 << max(0, int(np.ceil(np.log2(max(n, 1)))))
    return max(TA_MIN_DFT, size)


def ta_max_samples(numerology, dft_size, stride):
    """Half the normal CP (144 kappa / 2^(mu + 1)) in samples at dft_size x SCS x stride (estimate_ta_correlation,
    time_alignment_estimator_dft_impl.cpp:236)."""
    t_c = 1.0 / (480000 * 4096)
    half_cp = (144 * 64 // (1 << (numerology + 1))) * t_c
    fs = dft_size * (15 << numerology) * 1000.0 * stride
    return int(np.floor(half_cp * fs)), fs


def fractional_sample_delay(c):
    """time_alignment_estimator_dft_impl.cpp:51: quadratic fit over 3 or 5 correlation samples around the peak."""
    if c.size == 5:
        num = np.dot([-0.4, -0.2, 0.0, 0.2, 0.4], c)
        den = np.dot([0.571429, -0.285714, -0.571429, -0.285714, 0.571429], c)
        corr = 1.0
    else:
        num = np.dot([-0.5, 0.0, 0.5], c)
        den = np.dot([0.5, -1.0, 0.5], c)
        corr = 0.5
    with np.errstate(divide="ignore", invalid="ignore"):
        r = -corr * num / den
    if not np.isfinite(r) or abs(r) > 1.0:
        return 0.0
    return float(r)


def estimate_ta(planes, positions, numerology, stride):
    """time_alignment_estimator_dft_impl::estimate of the smoothed LSE planes (port_channel_estimator_helpers.cpp:246):
    type 1 (stride-2 pattern) copies the pilots to the first bins; otherwise the pilots go to their subcarrier offset
    from the lowest one (mask path, stride 1). Inverse DFT, |.|^2 summed over planes, peak within +-half CP, fractional
    refinement unless the DFT is the largest one. Returns seconds, rounded to Tc like phy_time_unit::from_seconds."""
    span = positions[-1] - positions[0] + 1 if stride == 1 else len(positions)
    M = ta_dft_size(span)
    corr = np.zeros(M)
    for f in planes:
        x = np.zeros(M, np.complex128)
        if stride == 1:
            x[positions - positions[0]] = f
        else:
            x[: f.size] = f
        corr += np.abs(np.fft.ifft(x) * M) ** 2
    m, fs = ta_max_samples(numerology, M, stride)
    d_i = int(np.argmax(corr[:m]))
    a_i = int(np.argmax(corr[M - m:]))
    idx = d_i if corr[d_i] >= corr[M - m + a_i] else -(m - a_i)
    frac = 0.0
    if M != TA_MAX_DFT:
        n = 5 if m > 2 else 3
        frac = fractional_sample_delay(np.array([corr[(idx + i - n // 2) % M] for i in range(n)]))
    ta = np.float32((idx + frac) / fs)
    t_c = 1.0 / (480000 * 4096)
    tc10 = int(float(ta) / t_c * 10.0)  # from_seconds: truncate x10, round half away
    tc = int(tc10 / 10) + int(np.fmod(tc10, 10) / 5)
    return tc * t_c


def td_interpolate(planes, dmrs_syms, first, last, l):
    """apply_td_domain_strategy, "interpolate" (port_channel_estimator_average_impl.cpp:509): linear in time between
    the DM-RS symbols around l, extrapolated from the first / last two."""
    before = max([d for d in dmrs_syms if first <= d < l], default=-1)
    after = min([d for d in dmrs_syms if l <= d < last], default=-1)
    if before == -1:
        second = min([d for d in dmrs_syms if after + 1 <= d < last], default=-1)
        if second == -1:
            return planes[0]
        before, after = after, second
    if after == -1:
        second_last = max([d for d in dmrs_syms if first <= d < before], default=-1)
        if second_last == -1:
            return planes[-1]
        before, after = second_last, before
    w = (l - before) / (after - before)
    i = sum(1 for d in dmrs_syms if first <= d < before)
    return planes[i] + (planes[i + 1] - planes[i]) * w


def estimate(cfg, grid, fd="filter", td="average", compensate_cfo=False, numerology=1, crb_mask=None,
             low_papr_id=None):
    """cfg: slot, scrambling_id, n_scid, dmrs_type2, scaling (beta), dmrs_symbol_mask, start_symbol, nof_symbols,
    rb_start, nof_rb, nof_rx_ports. grid (P, 14, nsc) complex. Returns (ch (P, 14, nsc) complex128 filled on the
    allocation, noise_var (P,), rsrp (P,), epre (P,), extra) with extra = dict(cfo_hz (P,) NaN when one DM-RS symbol,
    ta_s (P,), cfo_phase (P,) arg between the first two DM-RS symbols or None).

    CFO (preprocess_pilots_and_estimate_cfo, port_channel_estimator_average_impl.cpp:322): phase of
    sum lse_1 conj(lse_0) over the time between the first two DM-RS symbols' starts; with compensate_cfo every DM-RS
    symbol's LSE is derotated by its start epoch before combining, the noise residual re-rotates the prediction (:475)
    and every symbol's estimate is rotated by its epoch (:128).

    crb_mask (rb_mask, one byte per grid CRB) replaces the contiguous allocation: the pilots of the allocated CRBs are
    concatenated, smoothed and interpolated as one band (compute_hop :245-275, the filter sized by the CRB count), the
    time alignment takes the RE-mask path (pilots at their subcarrier offsets, port_channel_estimator_helpers.cpp:285),
    and PRB i of the interpolated band is the estimate of the i-th allocated CRB. (The reference writes every PRB of a
    non-contiguous mask at the lowest CRB instead, :297 -- a defect: tests/test_oracle_vs_reference.py pins the
    restatement against what it does write.)"""
    P = cfg["nof_rx_ports"]
    t2 = cfg["dmrs_type2"]
    beta = cfg["scaling"]
    pat = layer0_pattern(t2)
    offset, stride = pat[0], pat[1] - pat[0]
    rb0, nrb = cfg["rb_start"], cfg["nof_rb"]
    rbs = list(range(rb0, rb0 + nrb)) if crb_mask is None else [int(i) for i in np.flatnonzero(crb_mask)]
    contiguous = rbs[-1] - rbs[0] + 1 == len(rbs)
    nrb = len(rbs)
    sc = np.array([rb * 12 + k for rb in rbs for k in pat])
    first, last = cfg["start_symbol"], cfg["start_symbol"] + cfg["nof_symbols"]
    syms = [l for l in range(first, last) if (cfg["dmrs_symbol_mask"] >> l) & 1]
    Dn = len(syms)
    N = sc.size
    if low_papr_id is not None:
        pil = [low_papr_sequence(low_papr_id % 30, len(rbs) * 6) for _ in syms]
    else:
        pil = [dmrs_sequence(cfg["slot"], l, cfg["scrambling_id"], cfg["n_scid"], t2, rb0, nrb, rbs) for l in syms]
    ep = symbol_start_epochs(numerology)
    scs_hz = (15 << numerology) * 1000.0
    nsc = grid.shape[2]
    ch = np.zeros((P, 14, nsc), np.complex128)
    nvar, rsrp, epre = np.zeros(P), np.zeros(P), np.zeros(P)
    cfo_hz, ta_s, cfo_ph = np.full(P, np.nan), np.zeros(P), [None] * P
    for p in range(P):
        rx = [grid[p, l, sc].astype(np.complex128) for l in syms]
        lse = [r * np.conj(q) for r, q in zip(rx, pil)]
        cfo = None
        if Dn > 1:  # :350-361
            cfo_ph[p] = float(np.angle(np.dot(np.conj(lse[0]), lse[1])))
            cfo = cfo_ph[p] / (2 * np.pi) / (ep[syms[1]] - ep[syms[0]])
            cfo_hz[p] = cfo * scs_hz
            if compensate_cfo:
                lse = [y * np.exp(-2j * np.pi * ep[l] * cfo) for y, l in zip(lse, syms)]
        planes = [sum(lse) / (beta * Dn)] if td == "average" else [y / beta for y in lse]
        planes = [fd_smoothing(f, nrb, stride, fd) for f in planes]
        Q = len(planes)
        epre[p] = sum(np.sum(np.abs(r) ** 2) for r in rx) / (N * Dn)
        rsrp[p] = sum(np.sum(np.abs(f) ** 2) for f in planes) * beta * beta * Dn / Q / (N * Dn)
        h = sum(planes) * beta / Q
        noise = 0.0
        for r, q, l in zip(rx, pil, syms):
            pred = h * q
            if compensate_cfo and cfo is not None:
                pred = pred * np.exp(2j * np.pi * ep[l] * cfo)
            noise += np.sum(np.abs(r - pred) ** 2)
        nvar[p] = max(rsrp[p] / 1e10, noise / (N * Dn - 1))
        ta_s[p] = estimate_ta(planes, sc, numerology, stride if contiguous else 1)
        frs = [interpolate(f, offset, stride, nrb * 12) for f in planes]
        for l in range(first, last):
            fr = frs[0] if td == "average" else td_interpolate(frs, syms, first, last, l)
            if compensate_cfo and cfo is not None:
                fr = fr * np.exp(2j * np.pi * ep[l] * cfo)
            for i, rb in enumerate(rbs):
                ch[p, l, rb * 12: (rb + 1) * 12] = fr[i * 12: (i + 1) * 12]
    return ch, nvar, rsrp, epre, dict(cfo_hz=cfo_hz, ta_s=ta_s, cfo_phase=cfo_ph)
