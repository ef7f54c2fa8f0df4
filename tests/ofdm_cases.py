"""OFDM test configurations and helpers shared by the oracle-vs-reference tests, the golden-fixture generator and the
GPU parity tests. TEST INFRASTRUCTURE ONLY."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import ofdm_oracle  # noqa: E402,F401

# (numerology, bw_rb, dft_size, extended CP, scale, center frequency, slot within the subframe, window offset)
CASES = [
    (1, 273, 4096, False, 1.0 / 64, 3.5e9, 0, 0),      # n78 100 MHz, 122.88 Msps
    (1, 273, 4096, False, 0.0123, 3.6e9, 1, 17),
    (1, 106, 2048, False, 0.05, 3.3e9, 1, 0),           # 40 MHz
    (0, 52, 1024, False, 0.1, 1.8e9, 0, 5),             # 10 MHz 15 kHz: symbols 0 and 7 carry the long CP
    (0, 25, 512, False, 0.2, 2.6e9, 0, 0),
    (2, 66, 1024, True, 0.3, 28e9, 2, 0),               # 60 kHz extended CP
    (2, 135, 2048, False, 0.07, 27e9, 3, 3),
    (1, 24, 512, False, 0.25, 3.5e9, 0, 0),
    (1, 10, 256, False, 1.0, 0.0, 1, 0),
    (3, 66, 1024, False, 0.3, 28e9, 5, 0),              # 120 kHz
    (1, 273, 8192, False, 1.0 / 128, 3.5e9, 0, 31),     # 245.76 Msps
    (0, 6, 128, False, 0.5, 1.9e9, 0, 0),               # 1.4 MHz-like grid, 1.92 Msps
    # 3 x 2^m sizes of the generic DFT (dft_processor_generic_impl.cpp:213-222)
    (1, 106, 1536, False, 0.05, 3.5e9, 0, 0),           # 40 MHz, 46.08 Msps
    (1, 217, 3072, False, 1.0 / 48, 3.6e9, 1, 9),       # 80 MHz, 92.16 Msps
    (0, 25, 384, False, 0.2, 2.1e9, 0, 0),              # 5 MHz 15 kHz, 5.76 Msps
    (0, 52, 768, False, 0.1, 1.8e9, 0, 3),              # 10 MHz 15 kHz, 11.52 Msps
    (2, 51, 768, False, 0.3, 28e9, 3, 0),               # 60 kHz
    (1, 273, 6144, False, 1.0 / 96, 3.5e9, 0, 20),      # 100 MHz, 184.32 Msps
    (1, 273, 4608, False, 1.0 / 72, 3.5e9, 1, 11),      # 100 MHz, 138.24 Msps (9 x 512: two radix-3 passes)
    # Sizes above one workgroup's LDS (dft_processor_generic_impl.cpp:224-230): the two-kernel split transform.
    (1, 273, 9216, False, 1.0 / 144, 3.5e9, 1, 40),     # 276.48 Msps (9 x 1024)
    (1, 273, 12288, False, 1.0 / 192, 3.6e9, 0, 0),     # 368.64 Msps (3 x 4096)
    (0, 270, 18432, False, 1.0 / 288, 2.1e9, 0, 7),     # 15 kHz, 276.48 Msps (9 x 2048)
    (2, 273, 24576, False, 1.0 / 384, 27e9, 3, 0),      # 60 kHz, 1474.56 Msps (3 x 8192)
    (2, 273, 36864, False, 1.0 / 576, 28e9, 3, 100),    # 60 kHz (9 x 4096)
    (2, 135, 49152, True, 1.0 / 768, 28e9, 2, 0),       # 60 kHz extended CP (6 x 8192)
    (1, 273, 98304, False, 1.0 / 1536, 3.5e9, 1, 300),  # 30 kHz (12 x 8192)
]
# 120 kHz with 36864 / 98304 points is not in the list: the reference computes the sampling rate in 32 bits
# (subcarrier_spacing.h:279, 120 kHz x 36864 > 2^32) and gets wrong cyclic prefixes there
# (tests/test_oracle_vs_reference.py::test_ofdm_reference_sampling_rate_overflow).


def random_grid(rng, P, ns, nsc, occupancy=1.0):
    """A bf16 grid of unit-power QPSK-like values (some REs empty)."""
    x = (rng.normal(size=(P, ns, nsc)) + 1j * rng.normal(size=(P, ns, nsc))) / np.sqrt(2)
    x[rng.random((P, ns, nsc)) > occupancy] = 0
    return ofdm_oracle.complex_to_bf16(x)


def rel_err(got, want):
    return float(np.max(np.abs(got - want)) / max(np.sqrt(np.mean(np.abs(want) ** 2)), 1e-30))


def bf16_ulp_diff(a_u16, b_u16):
    """Per-value distance in bf16 units in the last place (sign-magnitude ordering)."""
    def ordered(u):
        u = u.astype(np.int32)
        return np.where(u & 0x8000, -(u & 0x7FFF), u)
    return np.abs(ordered(a_u16) - ordered(b_u16))


def bf16_close(got_u16, want_u16, atol_rel_rms=1e-4):
    """Fraction of significant values (|want| > 1e-3 RMS) that differ, and whether every value is within one bf16 ulp (<= 2^-7 relative) of the other or
    within atol_rel_rms x RMS in absolute terms (values near zero, e.g. empty REs, carry only DFT rounding noise)."""
    a = ofdm_oracle.bf16_to_complex(got_u16)
    b = ofdm_oracle.bf16_to_complex(want_u16)
    rms = np.sqrt(np.mean(np.abs(b) ** 2))
    ok = True
    for pa, pb in ((a.real, b.real), (a.imag, b.imag)):
        ok &= bool(np.all(np.abs(pa - pb) <= np.maximum(np.abs(pb) * 2.0 ** -7, atol_rel_rms * rms)))
    significant = np.abs(b) > 1e-3 * rms
    differ = np.any(got_u16 != want_u16, axis=-1)
    return ok, float(np.mean(differ[significant]))
