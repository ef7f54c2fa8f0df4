"""How reproducible are the reference's own PUSCH LLRs? The reference's CMake builds at -march=native
(CMakeLists.txt:524), and its srsvec reductions change order with the SIMD width (dot_prod.cpp:36: 8 complex lanes
with AVX2, 16 with AVX-512) while GCC contracts products into FMAs differently per target. The same 273-PRB test-mode
slot (tests/ul273_cases.py) through the reference's dmrs_pusch_estimator + pusch_demodulator built twice from source
(oracle/build_ref.sh: AVX2 + FMA, and SRSREF_MARCH=x86-64-v4) gives estimates differing in a few bf16 words and LLRs
differing by up to three steps on a few of 314 496 bits; with the same estimates the two demodulators agree within
one step. This pins the tolerance of the GPU's 273-PRB LLR test (tests/test_ul273_llr_gpu.py) to the reference's own
build-to-build spread. TEST INFRASTRUCTURE ONLY (CPU)."""
import os

import numpy as np
import pytest

import ul273_cases as U
from oracle_lib import Reference

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
V4_SO = os.path.join(ROOT, "oracle", "_ref", "libsrsref_x86-64-v4.so")

# Tolerances shared with tests/test_ul273_llr_gpu.py.
MAX_STEPS = 3
MIN_WITHIN_ONE = 0.9999


@pytest.mark.skipif(not os.path.exists(V4_SO), reason="AVX-512 reference build absent (oracle/build_ref.sh)")
def test_reference_builds_differ_within_tolerance():
    a = Reference()
    if not a.has_avx512():
        pytest.skip("host CPU without AVX-512")
    b = Reference(V4_SO)
    worst = 0
    for seed in (1, 2, 3):
        cfg, dcfg, g = U.ul273_case(np.random.default_rng(seed), snr_db=26.0)
        ra = a.pusch_chest(cfg, g, 273, fd=2, td=0, compensate_cfo=True)
        rb = b.pusch_chest(cfg, g, 273, fd=2, td=0, compensate_cfo=True)
        la = a.pusch_demodulate(dcfg, g, ra[0], ra[1], 273)
        lb = b.pusch_demodulate(dcfg, g, rb[0], rb[1], 273)
        st = U.llr_stats(la, lb)
        assert st["max"] <= MAX_STEPS and st["within1"] >= MIN_WITHIN_ONE, (seed, st)
        # The same estimates and noise variances: the demodulators agree within one step.
        assert U.llr_stats(la, b.pusch_demodulate(dcfg, g, ra[0], ra[1], 273))["max"] <= 1
        worst = max(worst, st["max"])
    assert worst >= 2, "the reference's builds no longer differ by more than one step: tighten the GPU tolerance"
