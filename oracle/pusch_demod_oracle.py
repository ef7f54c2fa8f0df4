"""TEST INFRASTRUCTURE ONLY — numpy restatement ("oracle") of the srsRAN PUSCH demodulator: channel equalization,
soft demapping and descrambling of one transmission, in float32 (equalizer: the reference's scalar paths; demapper: its SIMD paths). Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, as the checker.

Pinned against the reference's own pusch_demodulator_impl (generic channel equalizer, demodulation mapper,
pseudo-random descrambler) and demodulation_mapper_impl built from its sources (oracle/ref/ref_pusch_demod.cpp in
oracle/_ref/libsrsref.so) by tests/test_oracle_vs_reference.py, and against tests/golden/pusch_demod.npz by
tests/test_golden.py. The reference's x86 build takes AVX2 paths with approximate reciprocals (_mm256_rcp_ps), so the
pinning is within a tolerance: LLRs equal or one quantisation step apart on a small fraction.

Reference files (under /root/reference/lib/phy/upper/):
  channel_processors/pusch/pusch_demodulator_impl.cpp:272  per OFDM symbol: data REs (DM-RS REs excluded on DM-RS
                                                           symbols), equalize, demap, descramble (c_init = rnti 2^15
                                                           + n_id), LLRs RE-major then layer then bit
  equalization/channel_equalizer_generic_impl.cpp:286      ZF / MMSE dispatch; noise variance = max over ports for
                                                           two layers; MMSE with one layer == ZF (:343)
  equalization/equalize_zf_1xn.h:128                        ZF 1 x N: matched filter, ports with an abnormal channel
                                                           or noise variance skipped, nvar = sum |h|^2 nv / (sum |h|^2)^2
  equalization/equalize_zf_2xn.h:180                        ZF 2 x N: 2x2 Gram inverse, nvar_l = nv |h_other|^2 / det
  channel_modulation/demodulation_mapper_qpsk.cpp:45        QPSK: 2 sqrt(2) x rcp(nv), range 24 (SIMD path)
  channel_modulation/demodulation_mapper_qam16.cpp:43       16QAM closed form, range 20 (SIMD path)
  channel_modulation/demodulation_mapper_qam64.cpp / _qam256.cpp:212  interval (slope, intercept) tables = max-log LLR
                                                           of the Gray PAM, range 20
  channel_modulation/avx2_helpers.h:121, :236               SIMD quantize (x 120 / range, clip, round half even) and
                                                           near-zero parts (|x| <= 1e-9) -> 0
"""
import numpy as np

LLR_MAX = 120
F = np.float32


def gold_sequence(c_init, n):
    """TS 38.211 section 5.2.1 Gold sequence c(0..n-1)."""
    Nc = 1600
    x1 = np.zeros(Nc + n + 31, np.uint8)
    x2 = np.zeros(Nc + n + 31, np.uint8)
    x1[0] = 1
    for i in range(31):
        x2[i] = (c_init >> i) & 1
    for k in range(Nc + n):
        x1[k + 31] = x1[k + 3] ^ x1[k]
        x2[k + 31] = x2[k + 3] ^ x2[k + 2] ^ x2[k + 1] ^ x2[k]
    return x1[Nc:Nc + n] ^ x2[Nc:Nc + n]


def constellation_levels(qm):
    """Per real-bit position k (stream bit 2k of a symbol): (levels with bit 0, levels with bit 1) of the Gray PAM in
    odd-integer units, as modulation_mapper_lut_impl.cpp:39 builds the constellation."""
    half = qm // 2
    sets = [(set(), set()) for _ in range(half)]
    for idx in range(1 << qm):
        real, off = 0, -1
        for j in range(half):
            real += off
            off *= 2
            real *= 1 if (idx >> (2 * j + 1)) & 1 else -1
        for k in range(half):
            bit = (idx >> (qm - 1 - 2 * k)) & 1  # stream bit 2k, MSB first
            sets[k][bit].add(real)
    return [(sorted(a), sorted(b)) for a, b in sets]


def interval_tables(qm):
    """Max-log piecewise-linear tables per bit pair: (width multiple (2 or 4), slopes (int, units of a),
    intercepts (int numerators over avg / 2)). Pieces of width 2a, merged pairwise where every pair is identical."""
    L = 1 << (qm // 2)
    out = []
    for x0s, x1s in constellation_levels(qm):
        slopes, inters = [], []
        for i in range(L):
            y = 2 * (i - L // 2) + 1
            x0 = min(x0s, key=lambda x: abs(y - x))
            x1 = min(x1s, key=lambda x: abs(y - x))
            slopes.append(2 * (x0 - x1))
            inters.append((x1 * x1 - x0 * x0) // 2)
        if all(slopes[2 * i] == slopes[2 * i + 1] and inters[2 * i] == inters[2 * i + 1] for i in range(L // 2)):
            out.append((4, slopes[::2], inters[::2]))
        else:
            out.append((2, slopes, inters))
    return out


def quantize(v, range_limit):
    """SIMD quantizer (avx2_helpers.h:121 quantize_ps, same in the AVX-512 / NEON helpers): scale by 120 / range,
    clip to +-120, round half to even."""
    x = (np.asarray(v, F) * F(LLR_MAX / range_limit)).astype(F)
    x = np.clip(x, F(-LLR_MAX), F(LLR_MAX))
    return np.round(x).astype(np.int8)


def demap(sym, nvar, qm):
    """Soft demapping of complex symbols (n,) with noise variances (n,) -> (n * qm,) int8 LLRs, as the reference's
    SIMD paths compute it (every symbol but a remainder of < 8 per call on AVX2 / AVX-512 / NEON): reciprocal noise
    1 / nv for nv > 0 else 0 (safe_div), l = f(x) * rcp, and for 16/64/256QAM a real or imaginary part with
    |x| <= 1e-9 gives zero LLRs (avx2_helpers.h:250)."""
    sym = np.asarray(sym, np.complex64)
    nvar = np.asarray(nvar, F)
    n = sym.size
    re, im = sym.real.astype(F), sym.imag.astype(F)
    out = np.zeros((n, qm), np.int8)
    valid_nv = nvar > 0
    with np.errstate(divide="ignore"):
        rcp = np.where(valid_nv, F(1) / np.where(valid_nv, nvar, 1), F(0)).astype(F)
    if qm == 2:
        g = F(2.0) * F(np.sqrt(F(2.0)))
        for k, x in enumerate((re, im)):
            out[:, k] = quantize((g * x).astype(F) * rcp, 24)
        return out.reshape(-1)
    if qm == 4:
        a = F(1.0) / np.sqrt(F(10.0))
        for k, x in enumerate((re, im)):
            f = (F(4) * a * x).astype(F)
            l01 = np.where(np.abs(x) > F(2) * a, (F(2) * f - np.copysign(F(0.8), x)).astype(F), f).astype(F)
            l23 = (F(0.8) - np.abs(f)).astype(F)
            nz = np.abs(x) <= F(1e-9)
            out[:, k] = np.where(nz, 0, quantize(l01 * rcp, 20))
            out[:, 2 + k] = np.where(nz, 0, quantize(l23 * rcp, 20))
        return out.reshape(-1)
    avg = {6: 42, 8: 170}[qm]
    a = F(1.0) / np.sqrt(F(avg))
    for kb, (wm, slopes, inters) in enumerate(interval_tables(qm)):
        inv_width = F(1) / F(wm / np.sqrt(float(avg)))  # float INTERVAL_WIDTH = wm * M_SQRT1_<avg>; scaled by its
        # reciprocal (demodulation_mapper_qam64.cpp:49, avx2_helpers.h:178)
        nint = len(slopes)
        sl = np.array([F(s) * a for s in slopes], F)
        ic = np.array([F(c) / F(avg // 2) for c in inters], F)
        for k, x in enumerate((re, im)):
            idx = np.clip(np.floor((x * inv_width).astype(F)).astype(np.int64) + nint // 2, 0, nint - 1)
            l = ((sl[idx] * x).astype(F) + ic[idx]).astype(F) * rcp
            out[:, 2 * kb + k] = np.where(np.abs(x) <= F(1e-9), 0, quantize(l, 20))
    return out.reshape(-1)


def _isnormal(x):
    x = np.asarray(x, F)
    return np.isfinite(x) & (np.abs(x) >= np.finfo(F).tiny)


def equalize(rx, H, noise_var, mmse=False):
    """rx (P, n) complex64 received REs, H (P, L, n) complex64 channel estimates, noise_var (P,) -> (eq (n, L)
    complex64, nvar (n, L) float32), following the reference's scalar ZF paths (L = 1: any P; L = 2: P = 2 or 4).
    MMSE with L = 1 is ZF (channel_equalizer_generic_impl.cpp:343); L > 2 and MMSE with L >= 2 are not implemented by
    the reference (equalize_mmse_* assert) and raise here."""
    P, L, n = H.shape
    nv = np.asarray(noise_var, F)
    rx = rx.astype(np.complex64)
    H = H.astype(np.complex64)
    if L == 1:
        ch_mod_sq = np.zeros(n, F)
        nvar_acc = np.zeros(n, F)
        re_out = np.zeros(n, np.complex64)
        for p in range(P):
            h = H[p, 0]
            norm = (h.real * h.real + h.imag * h.imag).astype(F)
            ok = _isnormal(norm) & bool(_isnormal(nv[p]) and nv[p] > 0)
            ch_mod_sq = np.where(ok, ch_mod_sq + norm, ch_mod_sq).astype(F)
            nvar_acc = np.where(ok, nvar_acc + norm * nv[p], nvar_acc).astype(F)
            prod = (rx[p] * np.conj(h)).astype(np.complex64)
            re_out = np.where(ok, re_out + prod, re_out).astype(np.complex64)
        d = ch_mod_sq  # tx_scaling = 1
        good = _isnormal(d) & _isnormal(nvar_acc)
        with np.errstate(divide="ignore", invalid="ignore"):
            rcp = (F(1) / np.where(good, d, 1)).astype(F)
        eq = np.where(good, re_out * rcp, 0).astype(np.complex64)
        nvar = np.where(good, nvar_acc * rcp * rcp, np.inf).astype(F)
        return eq[:, None], nvar[:, None]
    if L == 2 and not mmse and P in (2, 4):
        nve = F(np.max(nv))
        if not (_isnormal(nve) and nve >= 0):
            return np.zeros((n, 2), np.complex64), np.full((n, 2), np.inf, F)
        norm = [np.sum([(H[p, l].real ** 2 + H[p, l].imag ** 2).astype(F) for p in range(P)], axis=0).astype(F)
                for l in range(2)]
        xi = np.sum([np.conj(H[p, 0]) * H[p, 1] for p in range(P)], axis=0).astype(np.complex64)
        xi_mod_sq = (xi.real * xi.real + xi.imag * xi.imag).astype(F)
        mi = [np.sum([np.conj(H[p, l]) * rx[p] for p in range(P)], axis=0).astype(np.complex64) for l in range(2)]
        d_pinv = (norm[0] * norm[1] - xi_mod_sq).astype(F)
        good = _isnormal(d_pinv)
        with np.errstate(divide="ignore", invalid="ignore"):
            rcp = (F(1) / np.where(good, d_pinv, 1)).astype(F)
        e0 = ((norm[1] * mi[0] - xi * mi[1]) * rcp).astype(np.complex64)
        e1 = ((norm[0] * mi[1] - np.conj(xi) * mi[0]) * rcp).astype(np.complex64)
        n0 = (nve * norm[1] * rcp).astype(F)
        n1 = (nve * norm[0] * rcp).astype(F)
        eq = np.stack([np.where(good, e0, 0), np.where(good, e1, 0)], axis=1).astype(np.complex64)
        nvar = np.stack([np.where(good, n0, np.inf), np.where(good, n1, np.inf)], axis=1).astype(F)
        return eq, nvar
    raise NotImplementedError(f"the reference does not implement {'MMSE' if mmse else 'ZF'} {L} layers x {P} ports")


def equalize_mmse(rx, H, noise_var):
    """Extension beyond the reference (parity unpinned): linear MMSE for L layers, float64, unbiased output.
    A = H^H H + nv I, x = diag(G)^-1 A^-1 H^H y with G = I - nv A^-1, nvar_l = nv [A^-1]_ll / g_l;
    nv = max over ports (like the reference's multi-layer paths)."""
    P, L, n = H.shape
    nv = float(np.max(noise_var))
    eq = np.zeros((n, L), np.complex128)
    var = np.zeros((n, L))
    for i in range(n):
        h = H[:, :, i].astype(np.complex128)
        A = h.conj().T @ h + nv * np.eye(L)
        Ai = np.linalg.inv(A)
        x = Ai @ (h.conj().T @ rx[:, i].astype(np.complex128))
        g = 1 - nv * np.real(np.diag(Ai))
        eq[i] = x / g
        var[i] = nv * np.real(np.diag(Ai)) / g
    return eq, var


def data_res(start_symbol, nof_symbols, dmrs_symbol_mask, dmrs_type2, nof_cdm_groups_without_data, rb_start, nof_rb):
    """(symbol, subcarrier) of the data REs in demodulation order (symbol-major, ascending subcarrier)."""
    out = []
    for l in range(start_symbol, start_symbol + nof_symbols):
        dm = (dmrs_symbol_mask >> l) & 1
        for rb in range(rb_start, rb_start + nof_rb):
            for k in range(12):
                group = (k % 6) // 2 if dmrs_type2 else k % 2
                if dm and group < nof_cdm_groups_without_data:
                    continue
                out.append((l, rb * 12 + k))
    return out


def demodulate(cfg, grid, ch_est, noise_var, mmse=False):
    """cfg dict (rnti, n_id, qm, nof_layers, nof_rx_ports, start_symbol, nof_symbols, dmrs_symbol_mask, dmrs_type2,
    nof_cdm_groups_without_data, rb_start, nof_rb); grid (P, 14, nsc) complex64; ch_est (L, P, 14, nsc) complex64;
    noise_var (P,) -> descrambled codeword LLRs (int8)."""
    res = data_res(cfg["start_symbol"], cfg["nof_symbols"], cfg["dmrs_symbol_mask"], cfg["dmrs_type2"],
                   cfg["nof_cdm_groups_without_data"], cfg["rb_start"], cfg["nof_rb"])
    sym = np.array([r[0] for r in res])
    sc = np.array([r[1] for r in res])
    P, L, qm = cfg["nof_rx_ports"], cfg["nof_layers"], cfg["qm"]
    rx = grid[:P, sym, sc]
    H = np.transpose(ch_est[:L, :P, sym, sc], (1, 0, 2))
    if L <= 2 and not (mmse and L == 2):
        eq, nvar = equalize(rx, H, noise_var, mmse)
    else:
        e, v = equalize_mmse(rx, H, noise_var)
        eq, nvar = e.astype(np.complex64), v.astype(F)
    llr = demap(eq.reshape(-1), nvar.reshape(-1), qm).astype(np.int16)
    c = gold_sequence(cfg["rnti"] * (1 << 15) + cfg["n_id"], llr.size)
    return np.where(c == 1, -llr, llr).astype(np.int8)


# ----------------------------------------------------------------------------------------------------------------------
# General allocations, transform precoding and post-equalization statistics (pusch_demodulator_impl.cpp:272-444).
# ----------------------------------------------------------------------------------------------------------------------

def allocated_rbs(rb_start, nof_rb, crb_mask=None):
    """CRBs of the allocation in ascending order: config.rb_mask (crb_mask, one byte per grid CRB) or the contiguous
    [rb_start, rb_start + nof_rb)."""
    if crb_mask is None:
        return list(range(rb_start, rb_start + nof_rb))
    return [int(i) for i in np.flatnonzero(np.asarray(crb_mask))]


def data_res_mask(start_symbol, nof_symbols, dmrs_symbol_mask, dmrs_type2, nof_cdm_groups_without_data, rbs):
    """As data_res over an arbitrary CRB list: re_mask = rb_mask kron active REs per PRB (pusch_demodulator_impl.cpp:
    290), symbol-major, ascending subcarrier."""
    out = []
    for l in range(start_symbol, start_symbol + nof_symbols):
        dm = (dmrs_symbol_mask >> l) & 1
        for rb in rbs:
            for k in range(12):
                group = (k % 6) // 2 if dmrs_type2 else k % 2
                if dm and group < nof_cdm_groups_without_data:
                    continue
                out.append((l, rb * 12 + k))
    return out


def modulate_bits(bits, qm):
    """Hard bits (n * qm,) -> complex64 constellation points, TS 38.211 section 5.1 (modulation_mapper_lut_impl.cpp:39
    builds the same points: Gray PAM per component, amplitude 1 / sqrt(average power))."""
    b = np.asarray(bits, np.int64).reshape(-1, qm)
    half = qm // 2
    avg = {2: 2, 4: 10, 6: 42, 8: 170}[qm]

    def pam(cols):
        # s_j = 1 - 2 b_j: s0 (2^(h-1) - s2 (2^(h-2) - ... (2 - s_{2(h-1)})))
        s = [1 - 2 * b[:, c] for c in cols]
        if half == 1:
            return s[0]
        inner = 2 - s[half - 1]
        for j in range(half - 2, 0, -1):
            inner = (1 << (half - j)) - s[j] * inner
        return s[0] * inner

    re = pam([2 * j for j in range(half)])
    im = pam([2 * j + 1 for j in range(half)])
    a = F(1) / np.sqrt(F(avg))
    return (re.astype(F) * a + 1j * (im.astype(F) * a)).astype(np.complex64)


def transform_deprecode(eq, nvar):
    """transform_precoder_dft_impl.cpp deprecode_ofdm_symbol (inverse DFT of the M_sc data REs, scaled 1 / sqrt(M_sc))
    and deprecode_ofdm_symbol_noise (every valid noise variance -- positive, finite -- replaced by their mean)."""
    m = eq.size
    x = (np.fft.ifft(eq.astype(np.complex128)) * m / np.sqrt(m)).astype(np.complex64)
    v = np.asarray(nvar, F)
    valid = (v > 0) & np.isfinite(v)
    mean = F(np.sum(v[valid], dtype=np.float64) / max(int(valid.sum()), 1)) if valid.any() else F(0)
    return x, np.where(valid, mean, v).astype(F)


def demodulate_ex(cfg, grid, ch_est, noise_var, mmse=False, crb_mask=None, transform_precoding=False,
                  nvars_out=None):
    """pusch_demodulator_impl::demodulate with a general CRB mask, transform precoding (one layer) and the
    post-equalization statistics. Returns (descrambled LLRs int8, stats (15, 2) float64: per OFDM symbol and, in row
    14, for the whole transmission, (post-equalization SINR dB, EVM); NaN rows for symbols without data).

    Statistics (:355-:443): SINR = -10 log10(mean of the equalizer noise variances that are not infinite) or +inf with
    none; EVM of a symbol = sqrt(mean |modulate(hard(LLR)) - equalized|^2) over its REs x layers
    (evm_calculator_generic_impl.cpp; hard bit = LLR <= 0, before descrambling), total = the per-symbol EVMs weighted
    by their sizes (filter_infinite_and_accumulate :225 skips the infinite values). nvars_out (a dict) receives each
    symbol's equalizer noise variances."""
    rbs = allocated_rbs(cfg["rb_start"], cfg["nof_rb"], crb_mask)
    P, L, qm = cfg["nof_rx_ports"], cfg["nof_layers"], cfg["qm"]
    llrs = []
    stats = np.full((15, 2), np.nan)
    tot_nv, tot_cnt, tot_evm, tot_n = 0.0, 0, 0.0, 0
    for l in range(cfg["start_symbol"], cfg["start_symbol"] + cfg["nof_symbols"]):
        res = data_res_mask(l, 1, cfg["dmrs_symbol_mask"], cfg["dmrs_type2"], cfg["nof_cdm_groups_without_data"], rbs)
        if not res:
            continue
        sc = np.array([r[1] for r in res])
        rx = grid[:P, l, sc]
        H = np.transpose(ch_est[:L, :P, l, sc], (1, 0, 2))
        if L <= 2 and not (mmse and L == 2):
            eq, nvar = equalize(rx, H, noise_var, mmse)
        else:
            e, v = equalize_mmse(rx, H, noise_var)
            eq, nvar = e.astype(np.complex64), v.astype(F)
        eq, nvar = eq.reshape(-1), nvar.reshape(-1)
        if transform_precoding:
            assert L == 1
            eq, nvar = transform_deprecode(eq, nvar)
        if nvars_out is not None:
            nvars_out[l] = nvar
        fin = ~np.isinf(nvar)
        s_nv, s_cnt = float(np.sum(nvar[fin], dtype=np.float64)), int(fin.sum())
        llr = demap(eq, nvar, qm)
        err = modulate_bits((llr <= 0).astype(np.uint8), qm) - eq
        e2 = float(np.sum(err.real.astype(np.float64) ** 2 + err.imag.astype(np.float64) ** 2))
        evm = np.sqrt(e2 / eq.size)
        stats[l] = (-10 * np.log10(s_nv / s_cnt) if s_cnt and s_nv > 0 else np.inf, evm)
        tot_nv, tot_cnt, tot_evm, tot_n = tot_nv + s_nv, tot_cnt + s_cnt, tot_evm + eq.size * evm, tot_n + eq.size
        llrs.append(llr)
    llr = np.concatenate(llrs).astype(np.int16) if llrs else np.zeros(0, np.int16)
    c = gold_sequence(cfg["rnti"] * (1 << 15) + cfg["n_id"], llr.size)
    if tot_n:
        stats[14] = (-10 * np.log10(tot_nv / tot_cnt) if tot_cnt and tot_nv > 0 else np.inf, tot_evm / tot_n)
    return np.where(c == 1, -llr, llr).astype(np.int8), stats
