"""Pins the CPU oracle (and the host SCH logic) against the fixtures the reference produced (tests/golden/, made by
tools/gen_golden.py from the reference built from its own sources). Runs everywhere, no reference tree needed."""
import numpy as np
import pytest

import golden_lib as G
from oracle_lib import Oracle
from srsgpu import sch


@pytest.fixture(scope="module")
def orc():
    return Oracle()


def test_crc_golden(orc):
    n = 0
    for poly, bits, want in G.crc_cases():
        assert orc.crc_bits(poly, bits) == want
        n += 1
    assert n == 30


def test_encoder_golden(orc):
    for bg, Z, msg, cb in G.encoder_cases():
        assert np.array_equal(orc.ldpc_encode(bg, Z, msg), cb), (bg, Z)


def test_decoder_golden(orc):
    nsucc = nfail = 0
    for c in G.decoder_cases():
        r, bits = orc.ldpc_decode(c["impl"], c["bg"], c["Z"], c["llr"], nof_crc_bits=c["nof_crc_bits"],
                                  nof_filler=c["filler"], crc_poly=c["crc_poly"], max_iter=c["max_iter"], scaling=0.8)
        assert r == c["iters"], c["Z"]
        assert np.array_equal(bits, c["bits"])
        nsucc += r >= 0
        nfail += r < 0
    assert nsucc > 20 and nfail > 20


def test_rate_matching_golden(orc):
    for c in G.rate_matching_cases():
        cb = orc.ldpc_encode(c["bg"], c["Z"], c["msg"])
        out = orc.rate_match(c["bg"], c["Z"], c["rv"], c["qm"], c["Nref"], c["filler"], cb, c["E"])
        assert np.array_equal(out, c["rm_out"])
        for (new_data, impl), want in c["dm_out"].items():
            got = orc.rate_dematch(impl, c["bg"], c["Z"], c["rv"], c["qm"], c["Nref"], c["filler"], new_data,
                                   c["dm_llr"], c["dm_init"])
            assert np.array_equal(got, want), (c["Z"], c["rv"], new_data, impl)


def oracle_pdsch_encode(orc, tb, bg, rv, qm, nof_layers, Nref, nof_ch_symbols):
    """Composes the oracle stages like pdsch_encoder_impl::encode (pdsch_encoder_impl.cpp:28) with the host
    segmentation (srsgpu.sch): TB CRC, segmentation, CB CRC24B, LDPC encoding, rate matching."""
    tbs = tb.size * 8
    seg = sch.segment(tbs, bg, qm, nof_layers, nof_ch_symbols)
    tb_bits = np.unpackbits(tb)
    tb_crc = orc.crc_bytes(sch.CRC24A if False else (3 if tbs <= 3824 else 0), tb)
    crc_bits = np.array([(tb_crc >> (seg.nof_tb_crc_bits - 1 - i)) & 1 for i in range(seg.nof_tb_crc_bits)],
                        np.uint8)
    payload = np.concatenate([tb_bits, crc_bits])
    cw = []
    K = seg.segment_length
    for cb in seg.codeblocks:
        msg = np.zeros(K, np.uint8)
        data = payload[cb.tb_offset: cb.tb_offset + cb.nof_info_bits +
                       (seg.nof_tb_crc_bits if cb.index == seg.nof_segments - 1 else 0)]
        msg[:data.size] = data
        used = data.size + (seg.zero_pad if cb.index == seg.nof_segments - 1 else 0)
        if seg.cb_crc_bits:
            c = orc.crc_bits(1, msg[:used])
            msg[used:used + 24] = [(c >> (23 - i)) & 1 for i in range(24)]
        enc = orc.ldpc_encode(bg, seg.lifting_size, msg)
        cw.append(orc.rate_match(bg, seg.lifting_size, rv, qm, Nref, seg.nof_filler_bits, enc, cb.rm_length))
    return np.concatenate(cw), seg


def test_pdsch_encoder_golden(orc):
    n = 0
    for c in G.pdsch_encoder_cases():
        cw, seg = oracle_pdsch_encode(orc, c["tb"], c["bg"], c["rv"], c["qm"], c["nof_layers"], c["Nref"],
                                      c["nof_ch_symbols"])
        assert seg.nof_segments == c["meta"].shape[0]
        assert np.array_equal(cw, c["cw"])
        n += 1
    assert n == 14
