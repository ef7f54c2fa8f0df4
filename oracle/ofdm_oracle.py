"""TEST INFRASTRUCTURE ONLY — numpy restatement ("oracle") of the srsRAN OFDM slot modulator and demodulator, in
complex128. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, as the checker.

Pinned against the reference's own ofdm_slot_modulator_impl / ofdm_slot_demodulator_impl with the generic DFT, built
from its sources (oracle/ref/ref_ofdm.cpp in oracle/_ref/libsrsref.so), by tests/test_oracle_vs_reference.py, and
against the committed reference outputs in tests/golden/ofdm.npz by tests/test_golden.py.

Reference files (under /root/reference/):
  lib/phy/lower/modulation/ofdm_modulator_impl.cpp:58     per symbol: grid lower half -> DFT bins [N - rg/2, N), upper
                                                           half -> bins [0, rg/2); inverse DFT (unnormalised,
                                                           dft_processor_generic_impl.cpp:205 sign +1); times
                                                           phase compensation * scale; cyclic prefix = last cp samples
  lib/phy/lower/modulation/ofdm_demodulator_impl.cpp:96   per symbol: N samples from cp_len - window_offset, direct
                                                           DFT, times phase compensation * scale, times the window
                                                           phase exp(j 2 pi offset k / N) (:79), bins back to the grid
  lib/phy/lower/modulation/phase_compensation_lut.h:50     coefficient of symbol s of the subframe:
                                                           exp(-+ j 2 pi f_c t_start(s)), t_start = CP-inclusive start
  include/srsran/ran/cyclic_prefix.h:93                   CP length in units of kappa: (144 >> mu) (+16 for symbols 0
                                                           and 7 * 2^mu of the subframe), extended: 512 >> mu
"""
import numpy as np


def cp_samples(numerology, dft_size, extended, symbol):
    """Cyclic prefix of symbol `symbol` of the subframe in samples (kappa units * 2^mu * N / 2048)."""
    if extended:
        units = 512 >> numerology
    else:
        units = 144 >> numerology
        if symbol == 0 or symbol == 7 * (1 << numerology):
            units += 16
    return units * (1 << numerology) * dft_size // 2048


def nsymb(extended):
    return 12 if extended else 14


def slot_size(numerology, dft_size, extended, slot):
    ns = nsymb(extended)
    return sum(cp_samples(numerology, dft_size, extended, ns * slot + l) + dft_size for l in range(ns))


def phase_coefficients(numerology, dft_size, extended, center_freq_hz, is_tx):
    """phase_compensation_lut: one complex64 coefficient per symbol of the subframe (computed in double)."""
    srate = 15e3 * (1 << numerology) * dft_size
    ns = nsymb(extended) * (1 << numerology)
    sign_two_pi = (-1.0 if is_tx else 1.0) * 2.0 * np.pi
    out, offset = [], 0
    for s in range(ns):
        offset += cp_samples(numerology, dft_size, extended, s)
        t = offset / srate
        out.append(np.complex64(np.exp(1j * sign_two_pi * center_freq_hz * t)))
        offset += dft_size
    return np.array(out, np.complex64)


def bf16_to_complex(grid_u16):
    """(..., 2) uint16 bf16 bit patterns -> complex128."""
    f = (grid_u16.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    return f[..., 0] + 1j * f[..., 1]


def complex_to_bf16(x):
    """complex -> (..., 2) uint16 bf16 bit patterns, float32 then round half to even (bf16.h:39)."""
    f = np.stack([np.real(x), np.imag(x)], axis=-1).astype(np.float32)
    u = f.view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def modulate(grid_u16, numerology, bw_rb, dft_size, extended, scale, center_freq_hz, slot):
    """grid (P, nsymb, 12 bw_rb, 2) bf16 -> (P, slot_size) complex128 time samples of slot `slot` of the subframe."""
    P, ns, nsc = grid_u16.shape[0], nsymb(extended), 12 * bw_rb
    X = bf16_to_complex(grid_u16)
    coef = phase_coefficients(numerology, dft_size, extended, center_freq_hz, True).astype(np.complex128)
    out = []
    for p in range(P):
        parts = []
        for l in range(ns):
            s = ns * slot + l
            b = np.zeros(dft_size, np.complex128)
            b[dft_size - nsc // 2:] = X[p, l, : nsc // 2]
            b[: nsc // 2] = X[p, l, nsc // 2:]
            x = np.fft.ifft(b) * dft_size * (coef[s] * np.float32(scale))
            cp = cp_samples(numerology, dft_size, extended, s)
            parts.append(np.concatenate([x[dft_size - cp:], x]))
        out.append(np.concatenate(parts))
    return np.array(out)


def demodulate(samples, numerology, bw_rb, dft_size, extended, scale, center_freq_hz, slot, window_offset=0):
    """(P, slot_size) complex time samples -> (P, nsymb, 12 bw_rb) complex128 grid values (before bf16 rounding)."""
    P, ns, nsc = samples.shape[0], nsymb(extended), 12 * bw_rb
    coef = phase_coefficients(numerology, dft_size, extended, center_freq_hz, False).astype(np.complex128)
    win = np.exp(1j * 2 * np.pi * window_offset * np.arange(dft_size) / dft_size) if window_offset else None
    grid = np.zeros((P, ns, nsc), np.complex128)
    for p in range(P):
        pos = 0
        for l in range(ns):
            s = ns * slot + l
            cp = cp_samples(numerology, dft_size, extended, s)
            x = samples[p, pos + cp - window_offset: pos + cp - window_offset + dft_size]
            y = np.fft.fft(x) * (coef[s] * np.float32(scale))
            if win is not None:
                y = y * win
            grid[p, l, : nsc // 2] = y[dft_size - nsc // 2:]
            grid[p, l, nsc // 2:] = y[: nsc // 2]
            pos += cp + dft_size
    return grid
