"""Pins the CPU restatement (oracle/liboracle.so) bit-for-bit against the srsRAN reference built from its own sources
(oracle/_ref/libsrsref.so). Skipped where the reference build is absent; tests/test_golden.py then pins the oracle
against the committed fixtures that tools/gen_golden.py generated from the same reference build.
"""
import numpy as np
import pytest

from oracle_lib import (BG_K, BG_N_SHORT, CRC16, CRC24A, CRC24B, CRC_LEN, LIFTING_SIZES, Oracle, Reference,
                        encode_with_llrs, have_ref)

pytestmark = [pytest.mark.ref, pytest.mark.skipif(not have_ref(), reason="reference build oracle/_ref absent")]


@pytest.fixture(scope="module")
def orc():
    return Oracle()


@pytest.fixture(scope="module")
def ref():
    return Reference()


def test_crc_all_polys(orc, ref):
    rng = np.random.default_rng(1)
    for poly in range(6):
        for n in [0, 1, 7, 8, 24, 100, 1000, 8448]:
            bits = rng.integers(0, 2, n).astype(np.uint8)
            assert orc.crc_bits(poly, bits) == ref.crc_bits(poly, bits), (poly, n)
        data = rng.integers(0, 256, 333).astype(np.uint8)
        assert orc.crc_bytes(poly, data) == ref.crc_bytes(poly, data)


@pytest.mark.parametrize("bg", [1, 2])
def test_encoder_all_lifting_sizes(orc, ref, bg):
    rng = np.random.default_rng(bg)
    for Z in LIFTING_SIZES:
        msg = rng.integers(0, 2, BG_K[bg] * Z).astype(np.uint8)
        want = ref.ldpc_encode(bg, Z, msg, impl=0)
        assert np.array_equal(orc.ldpc_encode(bg, Z, msg), want), Z
        assert np.array_equal(ref.ldpc_encode(bg, Z, msg, impl=1), want), Z


def _decode_cases():
    cases = []
    for bg in (1, 2):
        for Z in (2, 3, 5, 7, 9, 11, 13, 15, 16, 36, 52, 64, 104, 208, 240, 288, 320, 352, 384):
            cases.append((bg, Z))
    return cases


@pytest.mark.parametrize("bg,Z", _decode_cases())
def test_decoder_matches_reference(orc, ref, bg, Z):
    rng = np.random.default_rng(1000 * bg + Z)
    K, N = BG_K[bg], BG_N_SHORT[bg]
    impls = [(0, Reference.GENERIC), (1, Reference.AVX2)]
    if ref.has_avx512():
        impls.append((1, Reference.AVX512))
    for trial in range(4):
        noise = [0.0, 6.0, 9.0, 14.0][trial]
        crc_poly = CRC16 if trial % 2 == 0 else CRC24B
        nof_filler = 0 if trial < 2 else min(Z, (K - 2) * Z // 4)
        if K * Z - nof_filler < CRC_LEN[crc_poly] + 8:
            crc_poly = 5  # CRC6 for the tiniest codeblocks (the decoder's CRC is only used for early stopping)
        # Codeblock lengths: the minimum admissible, a ragged rate-matched one and the full one (multiples of Z).
        n_llr = [(K + 2) * Z, N * Z, (K + 7) * Z if bg == 1 else (K + 5) * Z, N * Z][trial]
        _, _, llr = encode_with_llrs(orc, rng, bg, Z, crc_poly=crc_poly, nof_filler=nof_filler, amp=12,
                                     noise=noise, n_llr=n_llr)
        for use_crc in (True, False):
            for mode, impl in impls:
                kw = dict(nof_crc_bits=16 if CRC_LEN[crc_poly] < 24 else 24, nof_filler=nof_filler,
                          crc_poly=crc_poly if use_crc else -1, max_iter=8, scaling=0.8)
                r_ref, o_ref = ref.ldpc_decode(impl, bg, Z, llr, **kw)
                r_orc, o_orc = orc.ldpc_decode(mode, bg, Z, llr, **kw)
                assert r_orc == r_ref, (trial, use_crc, impl)
                assert np.array_equal(o_orc, o_ref), (trial, use_crc, impl)


def test_decoder_random_llrs_and_trimmed_input(orc, ref):
    """Random +/-10 LLRs (the reference benchmark's input, tests/benchmarks/phy/upper/channel_coding/ldpc/
    ldpc_decoder_benchmark.cpp:129) and inputs whose tail is zero (trimmed by decode)."""
    rng = np.random.default_rng(7)
    for bg, Z in ((1, 384), (2, 384), (1, 24), (2, 10)):
        K, N = BG_K[bg], BG_N_SHORT[bg]
        llr = ((rng.integers(0, 2, N * Z) * 20) - 10).astype(np.int8)
        for mode, impl in ((0, 0), (1, 1)):
            r1, o1 = ref.ldpc_decode(impl, bg, Z, llr, max_iter=6)
            r2, o2 = orc.ldpc_decode(mode, bg, Z, llr, max_iter=6)
            assert r1 == r2 and np.array_equal(o1, o2)
        # Zero tail: only K*Z + 3Z significant LLRs.
        llr2 = llr.copy()
        llr2[(K + 3) * Z:] = 0
        for mode, impl in ((0, 0), (1, 1)):
            r1, o1 = ref.ldpc_decode(impl, bg, Z, llr2, max_iter=5, crc_poly=CRC16)
            r2, o2 = orc.ldpc_decode(mode, bg, Z, llr2, max_iter=5, crc_poly=CRC16)
            assert r1 == r2 and np.array_equal(o1, o2)
        # Too few significant LLRs: decode refuses (output all ones without CRC).
        llr3 = llr.copy()
        llr3[K * Z - 5:] = 0
        r1, o1 = ref.ldpc_decode(1, bg, Z, llr3)
        r2, o2 = orc.ldpc_decode(1, bg, Z, llr3)
        assert r1 == r2 == -1 and np.array_equal(o1, o2) and o1.all()


def test_decoder_scaling_factors(orc, ref):
    rng = np.random.default_rng(11)
    for sf in (0.5, 0.625, 0.75, 0.9, 0.99995):
        _, _, llr = encode_with_llrs(orc, rng, 1, 96, noise=8.0, amp=12)
        for mode, impl in ((0, 0), (1, 1)):
            r1, o1 = ref.ldpc_decode(impl, 1, 96, llr, crc_poly=CRC16, max_iter=10, scaling=sf)
            r2, o2 = orc.ldpc_decode(mode, 1, 96, llr, crc_poly=CRC16, max_iter=10, scaling=sf)
            assert r1 == r2 and np.array_equal(o1, o2), sf


def _rm_cases():
    rng = np.random.default_rng(3)
    cases = []
    for bg in (1, 2):
        for Z in (2, 13, 64, 208, 384):
            for rv in range(4):
                qm = [1, 2, 4, 6, 8][int(rng.integers(0, 5))]
                N = BG_N_SHORT[bg] * Z
                nsys = (BG_K[bg] - 2) * Z
                nof_filler = int(rng.integers(0, max(1, nsys // 3)))
                Nref = [0, int(N * 0.7)][int(rng.integers(0, 2))]
                E = qm * int(rng.integers(max(1, (BG_K[bg] * Z) // qm // 2), 3 * N // qm))
                cases.append((bg, Z, rv, qm, Nref, nof_filler, E))
    return cases


@pytest.mark.parametrize("case", _rm_cases())
def test_rate_match(orc, ref, case):
    bg, Z, rv, qm, Nref, nof_filler, E = case
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    K = BG_K[bg]
    msg = rng.integers(0, 2, K * Z).astype(np.uint8)
    msg[K * Z - nof_filler:] = 0  # filler bits are zeros in the encoder input (ldpc_segmenter_tx_impl.cpp:216)
    want = ref.rate_match(bg, Z, rv, qm, Nref, nof_filler, msg, E)
    cb = orc.ldpc_encode(bg, Z, msg)
    assert np.array_equal(orc.rate_match(bg, Z, rv, qm, Nref, nof_filler, cb, E), want)


@pytest.mark.parametrize("case", _rm_cases())
def test_rate_dematch(orc, ref, case):
    bg, Z, rv, qm, Nref, nof_filler, E = case
    rng = np.random.default_rng((hash(case) + 5) & 0xFFFF)
    N = BG_N_SHORT[bg] * Z
    llr = rng.integers(-120, 121, E).astype(np.int8)
    init = rng.integers(-120, 121, N).astype(np.int8)
    for new_data in (1, 0):
        for mode, impl in ((0, 0), (1, 1)):
            want = ref.rate_dematch(impl, bg, Z, rv, qm, Nref, nof_filler, new_data, llr, init)
            got = orc.rate_dematch(mode, bg, Z, rv, qm, Nref, nof_filler, new_data, llr, init)
            assert np.array_equal(got, want), (new_data, mode)


@pytest.mark.parametrize("bg,Z,rv,qm,filler,frac", [(1, 16, 0, 2, 51, 0.6), (1, 64, 0, 8, 46, 0.8), (2, 64, 1, 1, 115, 0.3),
                                                    (1, 384, 3, 4, 100, 0.5), (2, 13, 2, 6, 0, 0.9)])
def test_rate_dematch_limited_buffer_short_input(orc, ref, bg, Z, rv, qm, filler, frac):
    """Limited-buffer rate matching (Ncb < N) with an input that ends in the first pass: the tail zeroing of
    allot_llrs (ldpc_rate_dematcher_impl.cpp:198) applies to the end of the full buffer."""
    rng = np.random.default_rng(Z + rv)
    N = BG_N_SHORT[bg] * Z
    Nref = int(N * 0.75)
    E = qm * max(1, int(Nref * frac) // qm)
    llr = rng.integers(-120, 121, E).astype(np.int8)
    init = rng.integers(-120, 121, N).astype(np.int8)
    for new_data in (1, 0):
        for mode, impl in ((0, 0), (1, 1)):
            want = ref.rate_dematch(impl, bg, Z, rv, qm, Nref, filler, new_data, llr, init)
            got = orc.rate_dematch(mode, bg, Z, rv, qm, Nref, filler, new_data, llr, init)
            assert np.array_equal(got, want), (new_data, mode)


def test_pdsch_modulator_random(orc, ref):
    from pdsch_mod_cases import random_config
    rng = np.random.default_rng(77)
    for _ in range(80):
        cfg, nbits, w = random_config(rng, 40)
        cw = rng.integers(0, 256, (nbits + 7) // 8).astype(np.uint8)
        want = ref.pdsch_modulate(cfg, w, cw, nbits, 40)
        assert np.array_equal(orc.pdsch_modulate(cfg, w, cw, nbits, 40), want), cfg


def test_pdsch_modulator_full_band(orc, ref):
    from pdsch_mod_cases import full_band_config
    rng = np.random.default_rng(78)
    for L, qm in ((4, 8), (2, 6), (1, 2), (3, 4)):
        cfg, nbits = full_band_config(L, qm)
        w = (rng.normal(size=(4, L)) + 1j * rng.normal(size=(4, L))).astype(np.complex64)
        cw = rng.integers(0, 256, (nbits + 7) // 8).astype(np.uint8)
        want = ref.pdsch_modulate(cfg, w, cw, nbits, 273)
        assert np.array_equal(orc.pdsch_modulate(cfg, w, cw, nbits, 273), want), (L, qm)


def test_pdsch_modulator_general_vs_reference(orc, ref):
    """General allocations: type-0 VRB bitmaps mapped non-interleaved / interleaved (bundles 2, 4), reserved RE patterns
    and PRG precoding with one PRG over the grid (multi-PRG: see the next test). The reference's CRB mask
    (rb_allocation::get_crb_mask) equals the test-side restatement and the product's host mapping
    (srsgpu.alloc.vrb_to_crb_mask), and the oracle's grid over that mask equals the reference's grid bit for bit."""
    import srsgpu.alloc as A
    from oracle_lib import pdsch_modulate_general
    from pdsch_mod_cases import crb_mask_test_side, random_general_config
    rng = np.random.default_rng(79)
    G = 52
    for i in range(60):
        cfg, nbits, w = random_general_config(rng, G, interleave=[0, 2, 4][i % 3] if i < 30 else None,
                                              prg=[0, G][i % 2])
        cw = rng.integers(0, 256, (nbits + 7) // 8).astype(np.uint8)
        want, crb = pdsch_modulate_general(ref.lib, cfg, w, cw, nbits, G)
        assert np.array_equal(crb, crb_mask_test_side(cfg, G)), cfg
        il = cfg["interleave"]
        vtp = A.interleaved_other(cfg["bwp_start_rb"], cfg["bwp_size_rb"], il) if il else None
        assert np.array_equal(A.vrb_to_crb_mask(cfg["vrb_mask"], cfg["bwp_start_rb"], cfg["bwp_size_rb"], G, vtp), crb)
        got, _ = pdsch_modulate_general(orc.lib, cfg, w, cw, nbits, G, crb_mask=crb)
        assert np.array_equal(got, want), (i, cfg)


def test_pdsch_modulator_multi_prg_reference_defect(orc, ref):
    """Documents a reference defect instead of copying it: with more than one PRG, the symbol-buffer mapper the PDSCH
    modulator uses (resource_grid_mapper_impl.cpp:330-:340) adds the ABSOLUTE lowest active subcarrier
    (bounded_bitset::find_lowest returns absolute indexes) to the PRG's start, so PRG i > 0 starts at
    i * prg_size * 12 + lowest: REs of PRG 1.. are mapped with the wrong PRG's weights or not at all, and part of the
    codeword is silently dropped. The reference's own mapper test (resource_grid_mapper_test.cpp:270) and its pattern
    mapper (:220-:245) define the PRG of a RE as its subcarrier / (12 prg_size); the oracle and the GPU path implement
    that. This test pins (a) the defect (the reference maps fewer REs than the allocation holds) and (b) that the
    reference equals the oracle on PRG 0 of the first data symbol, before the first dropped RE shifts the codeword."""
    from oracle_lib import pdsch_modulate_general
    from pdsch_mod_cases import random_general_config
    rng = np.random.default_rng(80)
    G = 52
    for i in range(10):
        cfg, nbits, w = random_general_config(rng, G, interleave=0, prg=4, nof_reserved=0)
        cw = rng.integers(0, 256, (nbits + 7) // 8).astype(np.uint8)
        want, crb = pdsch_modulate_general(ref.lib, cfg, w, cw, nbits, G)
        got, _ = pdsch_modulate_general(orc.lib, cfg, w, cw, nbits, G, crb_mask=crb)
        mapped_ref = int((want[0] != 0).any(-1).sum())
        mapped_orc = int((got[0] != 0).any(-1).sum())
        if crb[4:].any():
            assert mapped_ref < mapped_orc, cfg
        l0 = int(np.flatnonzero((got[0] != 0).any(-1).any(-1))[0])
        assert np.array_equal(got[:, l0, :48], want[:, l0, :48]), cfg


@pytest.mark.parametrize("case", range(26))
def test_ofdm_oracle_vs_reference(ref, case):
    """OFDM modulator and demodulator restatement (oracle/ofdm_oracle.py, complex128) against the reference's
    ofdm_slot_modulator_impl / ofdm_slot_demodulator_impl with its generic float DFT: slot sizes equal, modulated
    samples within 2e-5 of the RMS (the reference's float radix-2 DFT error), demodulated bf16 grids equal except for
    1-ulp rounding-boundary differences (and DFT noise on empty REs)."""
    import ofdm_oracle as O
    from ofdm_cases import CASES, bf16_close, random_grid, rel_err
    mu, rb, N, ext, scale, fc, slot, woff = CASES[case]
    rng = np.random.default_rng(100 + case)
    ns = 12 if ext else 14
    assert ref.ofdm_slot_size(mu, rb, N, ext, slot) == O.slot_size(mu, N, ext, slot)
    grid = random_grid(rng, 2, ns, 12 * rb, occupancy=0.9)
    want = ref.ofdm_modulate(grid, mu, rb, N, ext, scale, fc, slot)
    got = O.modulate(grid, mu, rb, N, ext, scale, fc, slot)
    assert rel_err(got, want) < 2e-5
    # Demodulation of the reference's own samples.
    gref = ref.ofdm_demodulate(want, mu, rb, N, ext, 1.0 / (scale * N), fc, slot, woff)
    gorc = O.complex_to_bf16(O.demodulate(want.astype(np.complex128), mu, rb, N, ext, 1.0 / (scale * N), fc, slot,
                                          woff))
    # Above 8192 points the reference's own float error grows (its DFT-window phase ramp exp(j 2 pi woff b / N) is
    # evaluated in float for b up to N: ~1e-4 rad at 98304 points, woff 300): 3e-4 x RMS absolute there.
    ok, frac = bf16_close(gorc, gref, atol_rel_rms=1e-4 if N <= 8192 else 3e-4)
    assert ok and frac < 0.02, frac


def test_ofdm_reference_sampling_rate_overflow(ref):
    """Reference defect: to_sampling_rate_Hz<unsigned> (subcarrier_spacing.h:279) multiplies in 32 bits, so at 120 kHz
    the generic DFT's 36864- and 98304-point sizes overflow (4.42 / 11.8 GHz) and the slot is sized with wrong cyclic
    prefixes. The oracle (and the GPU plans) keep the TS 38.211 section 5.3.1 lengths; below 2^32 both agree."""
    import ofdm_oracle as O
    for mu, N, slot in ((3, 36864, 5), (3, 98304, 7)):
        assert 15000 * (1 << mu) * N >= 1 << 32
        assert ref.ofdm_slot_size(mu, 264, N, False, slot) != O.slot_size(mu, N, False, slot)
        cp = (144 >> mu) * (1 << mu) * N // 2048  # kappa units -> samples at N x scs
        assert O.slot_size(mu, N, False, slot) == 14 * (N + cp)
    assert ref.ofdm_slot_size(2, 264, 36864, False, 3) == O.slot_size(2, 36864, False, 3)


@pytest.mark.parametrize("qm", [2, 4, 6, 8])
def test_demapper_oracle_vs_reference(ref, qm):
    """Soft demapper restatement (max-log interval tables derived from the Gray PAM) against the reference's
    demodulation_mapper_impl: random symbols over +-1.5 x the constellation, near-zero symbols, noise variances
    including 0 and negative values. LLRs equal, or one quantisation step apart on < 1 %."""
    import pusch_demod_oracle as D
    rng = np.random.default_rng(qm)
    n = 20000
    x = ((rng.uniform(-1.5, 1.5, n) + 1j * rng.uniform(-1.5, 1.5, n))).astype(np.complex64)
    x[::97] = 0
    x[1::101] *= 1e-6
    nv = rng.uniform(0.001, 0.5, n).astype(np.float32)
    nv[::89] = 0
    nv[1::91] = -1
    want = ref.demodulate_soft(qm, x, nv).astype(np.int16)
    got = D.demap(x, nv, qm).astype(np.int16)
    d = np.abs(got - want)
    assert d.max() <= 1 and np.mean(d > 0) < 0.01, (d.max(), np.mean(d > 0))


@pytest.mark.parametrize("seed", range(12))
def test_pusch_demodulator_oracle_vs_reference(ref, seed):
    """Equalization (ZF 1 x 1..4, ZF 2 x 2 / 2 x 4, MMSE 1 layer) + demapping + descrambling restatement against the
    reference's pusch_demodulator_impl on random allocations, DM-RS patterns and channels. The reference's AVX2 path
    uses an approximate reciprocal: LLRs within one step, differing on < 5 %."""
    import pusch_demod_oracle as D
    from pusch_demod_cases import from_bf16, random_case
    rng = np.random.default_rng(300 + seed)
    cfg, grid, H, nv = random_case(rng, 24)
    mmse = bool(seed % 3 == 2 and cfg["nof_layers"] == 1)
    want = ref.pusch_demodulate(cfg, grid, H, nv, 24, mmse).astype(np.int16)
    got = D.demodulate(cfg, from_bf16(grid), from_bf16(H), nv, mmse).astype(np.int16)
    assert got.size == want.size
    d = np.abs(got - want)
    assert d.max() <= 1 and np.mean(d > 0) < 0.05, (cfg, d.max(), np.mean(d > 0))


@pytest.mark.parametrize("seed", range(16))
def test_pusch_demodulator_general_oracle_vs_reference(ref, seed):
    """General CRB masks, transform precoding (one layer; the reference's transform_precoder_dft_impl over exact DFTs,
    see oracle/ref/ref_pusch_demod.cpp) and the post-equalization statistics against the reference's
    pusch_demodulator_impl with the EVM calculator and SINR as the upper PHY builds it. LLRs within one step on < 5 %;
    EVM per symbol within 1e-2 relative (a hard decision flipped by the approximate reciprocal moves a small symbol's
    EVM by ~0.5 %), total within 5e-3, SINR within 5e-3 dB (the reference equalizer's approximate AVX2
    reciprocal moves each noise variance by ~1e-4, float sums run in a different order)."""
    import pusch_demod_oracle as D
    from pusch_demod_cases import from_bf16, random_general_case
    rng = np.random.default_rng(1300 + seed)
    tp = seed % 2 == 1
    cfg, grid, H, nv, crb = random_general_case(rng, 32, transform_precoding=tp, mask=seed % 3 != 2,
                                                max_rb=1 if seed % 4 == 0 else None)
    want, wstats = ref.pusch_demodulate_ex(cfg, grid, H, nv, 32, crb_mask=crb, transform_precoding=tp)
    got, gstats = D.demodulate_ex(cfg, from_bf16(grid), from_bf16(H), nv, crb_mask=crb, transform_precoding=tp)
    assert got.size == want.size
    d = np.abs(got.astype(np.int16) - want.astype(np.int16))
    assert d.max() <= 1 and np.mean(d > 0) < 0.05, (cfg, d.max(), np.mean(d > 0))
    assert np.array_equal(np.isnan(gstats), np.isnan(wstats))
    ok = ~np.isnan(wstats)
    np.testing.assert_allclose(gstats[:14, 1][ok[:14, 1]], wstats[:14, 1][ok[:14, 1]], rtol=1e-2)
    np.testing.assert_allclose(gstats[14, 1], wstats[14, 1], rtol=5e-3)
    # Two-layer ZF: the near-singular REs' noise variances dominate the mean and their 2 x 2 inverse is sensitive to
    # the rounding order (the reference: AVX2 with an approximate reciprocal), so 0.1 dB there.
    np.testing.assert_allclose(gstats[:, 0][ok[:, 0]], wstats[:, 0][ok[:, 0]],
                               atol=5e-3 if cfg["nof_layers"] == 1 else 0.1)


@pytest.mark.parametrize("seed", range(12))
def test_pusch_chest_crb_mask_oracle_vs_reference(ref, seed):
    """Non-contiguous CRB masks (rb_mask) against the reference's estimator: noise variance, RSRP, EPRE (1e-3
    relative), time alignment (2 Tc; RE-mask DFT path), CFO (0.05 Hz) are pinned as computed; the estimates are pinned
    through what the reference writes. Its write-back (port_channel_estimator_average_impl.cpp:295-304) puts every
    allocated PRB's 12 estimates at the lowest allocated CRB (the subspan never advances), so the reference's lowest
    CRB holds the LAST allocated PRB's estimate and every other allocated CRB stays unwritten (zero): the restatement's
    last-PRB estimate must equal the former (with the "average" time strategy; "interpolate" reads past the PRB's
    window, so only its metrics are pinned), and the restatement writes PRB i at CRB i of the mask (the intended
    mapping, which the GPU implements). Type 2 is left out: the reference's type-2 estimator is undefined behaviour in
    this build (see test_pusch_chest_type2_reference_is_undefined)."""
    import pusch_chest_oracle as C
    from ofdm_oracle import bf16_to_complex
    from pusch_chest_cases import random_case, random_crb_mask
    rng = np.random.default_rng(1500 + seed)
    mask = random_crb_mask(rng, 48, nof_rb=None)
    td = seed % 2
    comp = seed % 3 != 0
    cfg, grid, _ = random_case(rng, 48, crb_mask=mask, dmrs_type2=0,  # type 2: reference UB (see below)
                               cfo_hz=rng.uniform(-1500, 1500), delay=rng.uniform(-20, 20))
    ce, nv, rsrp, epre, ta, cfo = ref.pusch_chest(cfg, grid, 48, fd=2, td=td, compensate_cfo=comp, crb_mask=mask)
    ch, nv_o, rsrp_o, epre_o, ex = C.estimate(cfg, bf16_to_complex(grid), td="interpolate" if td else "average",
                                              compensate_cfo=comp, crb_mask=mask)
    np.testing.assert_allclose(nv, nv_o, rtol=1e-3)
    np.testing.assert_allclose(rsrp, rsrp_o, rtol=1e-3)
    np.testing.assert_allclose(epre, epre_o, rtol=1e-3)
    np.testing.assert_allclose(ta, ex["ta_s"], atol=2 * C.T_C if hasattr(C, "T_C") else 2 / (480000 * 4096))
    np.testing.assert_allclose(cfo, ex["cfo_hz"], atol=0.05)
    if td:
        return  # "interpolate" reads nof_re estimates from each PRB's 12-wide window: past it, undefined (:297)
    rbs = np.flatnonzero(mask)
    got = bf16_to_complex(ce)
    for l in range(cfg["start_symbol"], cfg["start_symbol"] + cfg["nof_symbols"]):
        want = ch[:, l, rbs[-1] * 12:(rbs[-1] + 1) * 12]
        g = got[:, l, rbs[0] * 12:(rbs[0] + 1) * 12]
        rms = np.sqrt(np.mean(np.abs(want) ** 2))
        assert np.max(np.abs(g - want)) < 2.5e-2 * rms, (cfg, l)
        assert not np.any(got[:, l, rbs[1] * 12:(rbs[1] + 1) * 12]), "the reference leaves the other CRBs unwritten"


@pytest.mark.parametrize("seed", range(12))
def test_pusch_chest_low_papr_oracle_vs_reference(ref, seed):
    """Transform-precoding DM-RS (low-PAPR sequence of group n_RS_ID mod 30: phase tables, the length-30 formula and
    Zadoff-Chu lengths, dmrs_pusch_estimator_impl.cpp:77) against the reference's estimator: estimates within
    1.5e-2 / 2.5e-2 x RMS, noise variance / RSRP / EPRE 1e-3, CFO 0.05 Hz, TA 2 Tc."""
    import pusch_chest_oracle as C
    from ofdm_oracle import bf16_to_complex
    from pusch_chest_cases import random_case
    from pusch_demod_cases import valid_tp_prbs
    rng = np.random.default_rng(1900 + seed)
    nrb = int(rng.choice([1, 2, 3, 4, 5] + valid_tp_prbs(48)[5:]))
    n_rs_id = int(rng.integers(0, 1008))
    td = seed % 2
    comp = seed % 3 != 0
    cfg, grid, _ = random_case(rng, 48, nof_rb=nrb, dmrs_type2=0, cfo_hz=rng.uniform(-1500, 1500),
                               delay=rng.uniform(-20, 20), low_papr_id=n_rs_id)
    ce, nv, rsrp, epre, ta, cfo = ref.pusch_chest(cfg, grid, 48, fd=2, td=td, compensate_cfo=comp,
                                                  low_papr_id=n_rs_id)
    ch, nv_o, rsrp_o, epre_o, ex = C.estimate(cfg, bf16_to_complex(grid), td="interpolate" if td else "average",
                                              compensate_cfo=comp, low_papr_id=n_rs_id)
    ls = slice(cfg["start_symbol"], cfg["start_symbol"] + cfg["nof_symbols"])
    ks = slice(cfg["rb_start"] * 12, (cfg["rb_start"] + cfg["nof_rb"]) * 12)
    got, want = bf16_to_complex(ce)[:, ls, ks], ch[:, ls, ks]
    assert np.max(np.abs(got - want)) < (2.5e-2 if td else 1.5e-2) * np.sqrt(np.mean(np.abs(want) ** 2)), cfg
    np.testing.assert_allclose(nv, nv_o, rtol=1e-3)
    np.testing.assert_allclose(rsrp, rsrp_o, rtol=1e-3)
    np.testing.assert_allclose(epre, epre_o, rtol=1e-3)
    np.testing.assert_allclose(ta, ex["ta_s"], atol=2 / (480000 * 4096))
    np.testing.assert_allclose(cfo, ex["cfo_hz"], atol=0.05)


@pytest.mark.parametrize("seed", range(24))
def test_pusch_chest_cfo_ta_oracle_vs_reference(ref, seed):
    """CFO estimation (compensated and not), time alignment and the interpolate time strategy of the restatement against
    the reference (1..100 RB, 1-3 DM-RS symbols, CFO up to 2 kHz, delays up to +-30 samples of a 4096-point DFT):
    estimates within 1.5e-2 (average) / 2.5e-2 (interpolate) x RMS, noise variance / RSRP 1e-3 relative, CFO within
    0.05 Hz, TA within 2 Tc."""
    import pusch_chest_oracle as C
    from ofdm_oracle import bf16_to_complex
    from pusch_chest_cases import random_case
    rng = np.random.default_rng(1000 + seed)
    nrb = [1, 2, 3, 4, 5, 24, 52, 100][seed % 8]
    gp = max(24, nrb + 3)
    td, comp, fd = seed % 2, (seed // 2) % 2, [2, 1, 0][(seed // 4) % 3]
    cfg, grid, _ = random_case(rng, gp, nof_rb=nrb, dmrs_type2=0, cfo_hz=rng.uniform(-2000, 2000),
                               delay=rng.uniform(-30, 30), snr_db=rng.uniform(5, 35))
    ce, nv, rsrp, epre, ta, cfo = ref.pusch_chest(cfg, grid, gp, fd=fd, td=td, compensate_cfo=comp)
    ch, nv_o, rsrp_o, epre_o, ex = C.estimate(cfg, bf16_to_complex(grid), ["none", "mean", "filter"][fd],
                                              ["average", "interpolate"][td], bool(comp))
    l0, l1 = cfg["start_symbol"], cfg["start_symbol"] + cfg["nof_symbols"]
    k0, k1 = cfg["rb_start"] * 12, (cfg["rb_start"] + nrb) * 12
    got, want = bf16_to_complex(ce)[:, l0:l1, k0:k1], ch[:, l0:l1, k0:k1]
    assert np.max(np.abs(got - want)) < [1.5e-2, 2.5e-2][td] * np.sqrt(np.mean(np.abs(want) ** 2))
    np.testing.assert_allclose(nv, nv_o, rtol=1e-3)
    np.testing.assert_allclose(rsrp, rsrp_o, rtol=1e-3)
    np.testing.assert_allclose(cfo, ex["cfo_hz"], atol=0.05)
    np.testing.assert_allclose(ta, ex["ta_s"], atol=2 / (480000 * 4096))


def test_pusch_chest_type2_reference_is_undefined(ref):
    """Type-2 PUSCH DM-RS in the reference is undefined behaviour, so it cannot pin type 2: configure_interpolator
    (port_channel_estimator_helpers.cpp:296) derives stride 1 from the type-2 RE pattern {0, 1, 6, 7}, so
    interpolator_linear_impl reads 12 x nof_rb values from a buffer of 4 x nof_rb pilots; with the "filter" smoothing and
    >= 2 RB filter_type (:83) also writes 2 x floor(nof_coefs / 2) + 1 > 15 tail-correction coefficients into its
    15-element array (the stack-smashing abort). Here, with "mean" smoothing (no filter_type), the reference returns
    estimates that are not the constant its own mean strategy computes."""
    from ofdm_oracle import bf16_to_complex
    from pusch_chest_cases import random_case
    rng = np.random.default_rng(4)
    cfg, grid, _ = random_case(rng, 24, nof_rb=4, dmrs_type2=1)
    ce = ref.pusch_chest(cfg, grid, 24, fd=1)[0]
    k0 = cfg["rb_start"] * 12
    row = bf16_to_complex(ce)[0, cfg["start_symbol"], k0:k0 + 48]
    assert not np.allclose(row, row[0], rtol=1e-2, atol=0)


@pytest.mark.parametrize("seed", range(14))
def test_pusch_chest_oracle_vs_reference(ref, seed):
    """DM-RS channel estimator restatement (float64) against the reference's dmrs_pusch_estimator_impl (float32, bf16
    output): estimates on the allocated REs within 1e-2 of the RMS channel magnitude, noise variance / RSRP / EPRE within
    1e-3 relative, for the filter (default), mean and none smoothing strategies and 1..24 RBs, DM-RS type 1 (type-2
    PUSCH DM-RS is undefined behaviour in the reference: test_pusch_chest_type2_reference_is_undefined)."""
    import pusch_chest_oracle as C
    from ofdm_oracle import bf16_to_complex
    from pusch_chest_cases import random_case
    rng = np.random.default_rng(400 + seed)
    nrb = [1, 2, 3, 4, 5, 24][seed % 6]
    cfg, grid, H = random_case(rng, 24, nof_rb=nrb, dmrs_type2=0)
    fd = ["filter", "mean", "none"][seed % 3] if seed >= 6 else "filter"
    ce, nv, rsrp, epre, ta, cfo = ref.pusch_chest(cfg, grid, 24, fd={"none": 0, "mean": 1, "filter": 2}[fd])
    ch, nv_o, rsrp_o, epre_o, _ = C.estimate(cfg, bf16_to_complex(grid), fd)
    l0, l1 = cfg["start_symbol"], cfg["start_symbol"] + cfg["nof_symbols"]
    k0, k1 = cfg["rb_start"] * 12, (cfg["rb_start"] + cfg["nof_rb"]) * 12
    got = bf16_to_complex(ce)[:, l0:l1, k0:k1]
    want = ch[:, l0:l1, k0:k1]
    rms = np.sqrt(np.mean(np.abs(want) ** 2))
    assert np.max(np.abs(got - want)) < 1e-2 * rms, (cfg, fd, np.max(np.abs(got - want)) / rms)
    np.testing.assert_allclose(nv, nv_o, rtol=1e-3)
    np.testing.assert_allclose(rsrp, rsrp_o, rtol=1e-3)
    np.testing.assert_allclose(epre, epre_o, rtol=1e-3)


@pytest.mark.parametrize("seed", range(10))
def test_pdsch_dmrs_oracle_vs_reference(ref, seed):
    """PDSCH DM-RS restatement bit-exact against the reference's dmrs_pdsch_processor_impl (1-4 layers and ports,
    DM-RS types 1 and 2, single and double symbols, reference point, amplitude)."""
    import pdsch_dmrs_oracle as M
    from pdsch_dmrs_cases import random_config
    rng = np.random.default_rng(500 + seed)
    cfg, w = random_config(rng, 24)
    assert np.array_equal(M.dmrs_map(cfg, w, 24), ref.dmrs_pdsch_map(cfg, w, 24)), cfg


@pytest.mark.parametrize("seed", range(10))
def test_pdsch_dmrs_crb_mask_oracle_vs_reference(ref, seed):
    """PDSCH DM-RS over a general CRB mask (rb_mask: RBG runs or scattered CRBs, the sequence skipping the gaps,
    dmrs_helper.cpp:64) bit-exact against the reference's dmrs_pdsch_processor_impl."""
    import pdsch_dmrs_oracle as M
    from pdsch_dmrs_cases import random_mask_config
    rng = np.random.default_rng(700 + seed)
    cfg, w, mask = random_mask_config(rng, 51)
    want = ref.dmrs_pdsch_map(cfg, w, 51, crb_mask=mask)
    assert np.array_equal(M.dmrs_map(cfg, w, 51, crb_mask=mask), want), cfg
    # A mask of exactly the contiguous allocation [rb_start, rb_start + nof_rb) reproduces the plain configuration.
    contiguous = np.zeros(51, np.uint8)
    contiguous[cfg["rb_start"]:cfg["rb_start"] + cfg["nof_rb"]] = 1
    assert np.array_equal(ref.dmrs_pdsch_map(cfg, w, 51, crb_mask=contiguous), ref.dmrs_pdsch_map(cfg, w, 51))


@pytest.mark.parametrize("seed", range(40))
def test_ulsch_demux_oracle_vs_reference(ref, seed):
    """UCI-on-PUSCH demultiplexing restatement bit-exact against the reference's ulsch_demultiplex_impl: random
    allocations / DM-RS patterns, HARQ-ACK of 0, 1, 2 (placeholders on the reserved REs, zeroed for the UL-SCH) or
    more bits, CSI Part 1 and CSI Part 2 (1- / 2-bit placeholders included), QPSK..256QAM, 1-2 layers, the codeword fed
    in odd-sized blocks."""
    import ulsch_demux_oracle as U
    from ulsch_demux_cases import nof_llrs, random_config
    rng = np.random.default_rng(1700 + seed)
    cfg, c2b, c2e, c_init = random_config(rng)
    llrs = rng.integers(-120, 121, nof_llrs(cfg)).astype(np.int8)
    want = ref.ulsch_demux(cfg, llrs, c_init, c2b, c2e, block_size=int(rng.integers(7, 500)))
    got = U.demultiplex(cfg, llrs, c_init, c2b, c2e)
    for k in ("sch", "harq", "csi1", "csi2"):
        assert np.array_equal(got[k], want[k]), (k, cfg, c2b, c2e)
    assert want["harq"].size == cfg["nof_enc_harq_ack_bits"] and want["csi2"].size == c2e


@pytest.mark.parametrize("seed", range(30))
def test_ulsch_demux_csi2_after_csi1_oracle_vs_reference(ref, seed):
    """CSI Part 2 placed where the reference's PUSCH processor configures it: set_csi_part2 runs when CSI Part 1 has
    been decoded, i.e. while the symbol completing CSI Part 1 is demultiplexed (pusch_processor_impl.cpp:72-100,
    ulsch_demultiplex_impl.cpp:241/:450), so CSI Part 2 takes REs of that symbol and the later ones only. The
    restatement with csi2_first_symbol = the CSI Part 1 end symbol (what the GPU batch's plan is given) equals the
    reference's demultiplexer driven that way."""
    import ulsch_demux_oracle as U
    from ulsch_demux_cases import nof_llrs, random_config
    rng = np.random.default_rng(4100 + seed)
    cfg, c2b, c2e, c_init = random_config(rng, csi2_after_csi1=True)
    llrs = rng.integers(-120, 121, nof_llrs(cfg)).astype(np.int8)
    want = ref.ulsch_demux(cfg, llrs, c_init, c2b, c2e, block_size=int(rng.integers(7, 500)), csi2_after_csi1=True)
    got = U.demultiplex(cfg, llrs, c_init, c2b, c2e, csi2_first_symbol=U.csi1_end_symbol(cfg) or 0)
    for k in ("sch", "harq", "csi1", "csi2"):
        assert np.array_equal(got[k], want[k]), (k, cfg, c2b, c2e)
    assert want["csi2"].size == c2e
