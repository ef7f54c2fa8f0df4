"""GPU parity of the LDPC decoder (HIP, through the C ABI) against the CPU oracle (itself pinned to the reference).
Bit-exact: decoded hard bits and the returned iteration count / failure must be identical."""
import numpy as np
import pytest

from oracle_lib import BG_K, BG_N_SHORT, CRC16, CRC24A, CRC24B, CRC_LEN, LIFTING_SIZES, Oracle, encode_with_llrs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def orc():
    return Oracle()


@pytest.fixture(scope="module")
def ctx():
    import srsgpu
    return srsgpu.Context(0)


# Kernel variants of the packed (even Z) decoder, forced through the context's kernel options (srsgpu_option,
# capi.cpp): the one-codeblock kernel, its edge-split variant and the two-codeblock workgroups (Z = 144..192).
VARIANTS = {"plain": dict(decoder_split=0, decoder_pairs=0),
            "split": dict(decoder_split=1, decoder_pairs=0),
            "pairs": dict(decoder_split=0, decoder_pairs=1)}


@pytest.fixture(params=sorted(VARIANTS))
def variant(request, ctx):
    with ctx.options(**VARIANTS[request.param]):
        yield request.param


def _case(orc, rng, bg, Z, trial):
    K, N = BG_K[bg], BG_N_SHORT[bg]
    noise = [0.0, 5.0, 8.0, 11.0, 16.0][trial % 5]
    crc_poly = [CRC16, CRC24B, CRC24A][trial % 3]
    nof_filler = 0 if trial % 2 == 0 else min(Z, (K - 2) * Z // 5)
    if K * Z - nof_filler < CRC_LEN[crc_poly] + 8:
        crc_poly = 5
    n_nodes = int(rng.integers(K + 2, N + 1))
    _, _, llr = encode_with_llrs(orc, rng, bg, Z, crc_poly=crc_poly, nof_filler=nof_filler, amp=12, noise=noise,
                                 n_llr=n_nodes * Z)
    return llr, crc_poly, nof_filler


@pytest.mark.parametrize("dec_type,mode", [("avx2", 1), ("generic", 0)])
def test_decoder_all_lifting_sizes_batched(orc, ctx, dec_type, mode, variant):
    """Every lifting size of both base graphs, mixed in ONE batch (one launch per base graph)."""
    import srsgpu
    rng = np.random.default_rng(2024 + mode)
    dec = srsgpu.LdpcDecoder(ctx, dec_type)
    llrs, cfgs, polys, want = [], [], [], []
    for bg in (1, 2):
        for Z in LIFTING_SIZES:
            for trial in range(3):
                llr, crc_poly, nof_filler = _case(orc, rng, bg, Z, trial + Z)
                use_crc = (trial != 2)
                cfg = srsgpu.CodeblockDecodeConfig(bg, Z, nof_crc_bits=16 if CRC_LEN[crc_poly] < 24 else 24,
                                                   nof_filler_bits=nof_filler, max_iterations=8)
                llrs.append(llr)
                cfgs.append(cfg)
                polys.append(crc_poly if use_crc else None)
                r, bits = orc.ldpc_decode(mode, bg, Z, llr, nof_crc_bits=cfg.nof_crc_bits, nof_filler=nof_filler,
                                          crc_poly=crc_poly if use_crc else -1, max_iter=8, scaling=0.8)
                want.append((None if r < 0 else r, bits))
    got = dec.decode_batch(llrs, cfgs, polys)
    n_success = 0
    for i, ((r_g, b_g), (r_w, b_w)) in enumerate(zip(got, want)):
        assert r_g == r_w, (i, cfgs[i], polys[i], r_g, r_w)
        assert np.array_equal(b_g, b_w), (i, cfgs[i], polys[i])
        n_success += r_w is not None
    assert n_success > len(want) // 3  # the batch exercises both early stops and failures


def test_decoder_bg1_z384_full_batch(orc, ctx, variant):
    """The benchmark shape (BG1, Z = 384): 256 codeblocks, several SNRs, 8 iterations with CRC24B early stop."""
    import srsgpu
    rng = np.random.default_rng(99)
    dec = srsgpu.LdpcDecoder(ctx, "auto")
    llrs, cfgs, polys, want = [], [], [], []
    for i in range(256):
        _, _, llr = encode_with_llrs(orc, rng, 1, 384, crc_poly=CRC24B, amp=10, noise=[4.0, 8.0, 10.0, 12.0][i % 4])
        cfg = srsgpu.CodeblockDecodeConfig(1, 384, nof_crc_bits=24, max_iterations=8)
        llrs.append(llr)
        cfgs.append(cfg)
        polys.append(CRC24B)
        r, bits = orc.ldpc_decode(1, 1, 384, llr, nof_crc_bits=24, crc_poly=CRC24B, max_iter=8)
        want.append((None if r < 0 else r, bits))
    got = dec.decode_batch(llrs, cfgs, polys)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g[0] == w[0] and np.array_equal(g[1], w[1]), i


def test_decoder_edge_cases(orc, ctx, variant):
    """Zero-tail trimming, too-short input (no decoding: all ones without CRC, untouched output with CRC), random
    +/-10 LLRs (the reference benchmark input) and scaling factors near the limits."""
    import srsgpu
    rng = np.random.default_rng(5)
    dec = srsgpu.LdpcDecoder(ctx, "avx2")
    for bg, Z in ((1, 384), (2, 384), (1, 24), (2, 10), (1, 2)):
        K, N = BG_K[bg], BG_N_SHORT[bg]
        llr = ((rng.integers(0, 2, N * Z) * 20) - 10).astype(np.int8)
        cfg = srsgpu.CodeblockDecodeConfig(bg, Z, max_iterations=6)
        r, b = dec.decode(llr, cfg)
        r0, b0 = orc.ldpc_decode(1, bg, Z, llr, max_iter=6)
        assert r is None and r0 == -1 and np.array_equal(b, b0)
        llr2 = llr.copy()
        llr2[(K + 3) * Z:] = 0
        r, b = dec.decode(llr2, cfg, crc_poly=CRC16)
        r0, b0 = orc.ldpc_decode(1, bg, Z, llr2, max_iter=6, crc_poly=CRC16)
        assert (r if r is not None else -1) == r0 and np.array_equal(b, b0)
        llr3 = llr.copy()
        llr3[K * Z - 5:] = 0
        r, b = dec.decode(llr3, cfg)
        assert r is None and b.all()
        init = rng.integers(0, 2, K * Z).astype(np.uint8)
        r, b = dec.decode(llr3, cfg, crc_poly=CRC16, output_init=init)
        assert r is None and np.array_equal(b, init)
    for sf in (0.5, 0.625, 0.75, 0.9, 0.99995):
        _, _, llr = encode_with_llrs(orc, rng, 1, 96, noise=8.0, amp=12)
        for dec_type, mode in (("generic", 0), ("avx2", 1)):
            d = srsgpu.LdpcDecoder(ctx, dec_type)
            r, b = d.decode(llr, srsgpu.CodeblockDecodeConfig(1, 96, max_iterations=10, scaling_factor=sf),
                            crc_poly=CRC16)
            r0, b0 = orc.ldpc_decode(mode, 1, 96, llr, crc_poly=CRC16, max_iter=10, scaling=sf)
            assert (r if r is not None else -1) == r0 and np.array_equal(b, b0), (sf, dec_type)


def test_decoder_rejects_invalid_configs(ctx):
    import srsgpu
    dec = srsgpu.LdpcDecoder(ctx, "avx2")
    llr = np.ones(66 * 17, np.int8)
    with pytest.raises(srsgpu.SrsGpuError):
        dec.decode(llr, srsgpu.CodeblockDecodeConfig(1, 17))  # invalid lifting size
    with pytest.raises(srsgpu.SrsGpuError):
        dec.decode(np.ones(66 * 16, np.int8), srsgpu.CodeblockDecodeConfig(1, 16, nof_crc_bits=11))
    with pytest.raises(srsgpu.SrsGpuError):
        dec.decode(np.ones(67 * 16, np.int8), srsgpu.CodeblockDecodeConfig(1, 16))  # too long
    with pytest.raises(srsgpu.SrsGpuError):
        dec.decode(np.ones(66 * 16, np.int8), srsgpu.CodeblockDecodeConfig(1, 16, scaling_factor=1.0))


def test_decoder_golden_vectors(ctx, variant):
    """The GPU decoder against the reference's own outputs (tests/golden/ldpc_decoder.npz), every case in one batch
    per arithmetic variant."""
    import golden_lib as G
    import srsgpu
    cases = list(G.decoder_cases())
    for impl, dec_type in ((0, "generic"), (1, "avx2")):
        sel = [c for c in cases if c["impl"] == impl]
        dec = srsgpu.LdpcDecoder(ctx, dec_type)
        cfgs = [srsgpu.CodeblockDecodeConfig(c["bg"], c["Z"], nof_crc_bits=c["nof_crc_bits"],
                                             nof_filler_bits=c["filler"], max_iterations=c["max_iter"]) for c in sel]
        got = dec.decode_batch([c["llr"] for c in sel], cfgs,
                               [None if c["crc_poly"] < 0 else c["crc_poly"] for c in sel])
        for c, (r, bits) in zip(sel, got):
            assert (r if r is not None else -1) == c["iters"], (c["bg"], c["Z"])
            assert np.array_equal(bits, c["bits"])


@pytest.mark.parametrize("mode", [1, 0])
def test_decoder_pairs_mixed_workgroups(orc, ctx, mode):
    """Two-codeblock workgroups (SRSGPU_OPTION_DECODER_PAIRS) with everything that differs between the slots of one
    workgroup: codeblocks that stop at different iterations or never, different layer counts (input lengths, trailing
    zeros), too-short inputs, mixed CRC polynomials and filler lengths, odd counts that leave a slot empty, at every
    lifting size the pairs take (Z = 144..192). Against the oracle, bit-exact."""
    import srsgpu
    with ctx.options(decoder_split=0, decoder_pairs=1):
        _pairs_mixed(orc, ctx, mode)


def _pairs_mixed(orc, ctx, mode):
    import srsgpu
    rng = np.random.default_rng(77 + mode)
    dec = srsgpu.LdpcDecoder(ctx, "avx2" if mode == 1 else "generic")
    llrs, cfgs, polys, want = [], [], [], []
    for bg, Z in ((1, 192), (1, 176), (2, 160), (2, 144), (1, 160)):
        K = BG_K[bg]
        for i in range(23):
            crc_poly = [CRC24B, CRC16, CRC24A][i % 3]
            nof_filler = 0 if i % 4 else min(Z, (K - 2) * Z // 7)
            n_nodes = K + 2 + int(rng.integers(1, 15))  # 8- and 16-layer classes
            _, _, llr = encode_with_llrs(orc, rng, bg, Z, crc_poly=crc_poly, nof_filler=nof_filler, amp=10,
                                         noise=[3.0, 6.0, 9.0, 12.0, 14.0][i % 5], n_llr=n_nodes * Z)
            if i % 7 == 3:
                llr[(n_nodes - 1) * Z:] = 0  # a trailing zero column: one layer fewer than the host bound
            if i % 11 == 5:
                llr[K * Z - 3:] = 0          # too short: no decoding
            cfg = srsgpu.CodeblockDecodeConfig(bg, Z, nof_crc_bits=16 if crc_poly == CRC16 else 24,
                                               nof_filler_bits=nof_filler, max_iterations=6)
            llrs.append(llr)
            cfgs.append(cfg)
            polys.append(crc_poly)
            r, bits = orc.ldpc_decode(mode, bg, Z, llr, nof_crc_bits=cfg.nof_crc_bits, nof_filler=nof_filler,
                                      crc_poly=crc_poly, max_iter=6, scaling=0.8)
            want.append((None if r < 0 else r, bits))
    got = dec.decode_batch(llrs, cfgs, polys)
    its = set()
    for i, ((r_g, b_g), (r_w, b_w)) in enumerate(zip(got, want)):
        assert r_g == r_w, (i, r_g, r_w)
        assert np.array_equal(b_g, b_w), i
        its.add(r_w)
    assert None in its and len(its) >= 4  # failures and several stop iterations within the batch
