"""GPU parity of the PDSCH encoder (TB CRC + segmentation + CB CRC + LDPC + rate matching, through the C ABI) against
the reference's own codewords (tests/golden/pdsch_encoder.npz) and the oracle composition on random grants."""
import numpy as np
import pytest

import golden_lib as G
from chain_lib import oracle_pdsch_encode
from oracle_lib import Oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import srsgpu
    return srsgpu.Context(0)


def test_pdsch_encoder_golden(ctx):
    import srsgpu
    enc = srsgpu.PdschEncoder(ctx)
    cases = list(G.pdsch_encoder_cases())
    cws = enc.encode_batch([c["tb"] for c in cases],
                           [srsgpu.PdschTransportBlock(c["bg"], c["rv"], c["qm"], c["nof_layers"], c["nof_ch_symbols"],
                                                       c["Nref"]) for c in cases])
    for c, cw in zip(cases, cws):
        assert np.array_equal(cw, c["cw"]), (c["bg"], c["rv"], c["qm"], c["nof_layers"])


def test_pdsch_encoder_random_grants(ctx):
    """200 random transport blocks (BG1/BG2, every rv and Qm, LBRM, 1-4 layers, TBS from 24 bits to ~100 kbit) in
    ONE plan, against the oracle composition."""
    import srsgpu
    from srsgpu import sch
    orc = Oracle()
    rng = np.random.default_rng(4)
    tbs, cfgs, want = [], [], []
    tables = list(sch.MCS_TABLE_256QAM.values())
    while len(cfgs) < 200:
        qm, r = tables[int(rng.integers(0, len(tables)))]
        g = sch.UeGrant(int(rng.integers(1, 60)), int(rng.integers(1, 5)), qm, r,
                        nof_symb_sh=int(rng.integers(4, 15)))
        seg = g.segmentation()
        rv = int(rng.integers(0, 4))
        N = (66 if seg.base_graph == 1 else 50) * seg.lifting_size
        nsys = ((22 if seg.base_graph == 1 else 10) - 2) * seg.lifting_size
        Nref = 0 if rng.integers(0, 3) else int(rng.integers(nsys + 1, N + 1))
        tb = rng.integers(0, 256, seg.tbs // 8).astype(np.uint8)
        cw, _, _ = oracle_pdsch_encode(orc, tb, seg.base_graph, rv, g.qm, g.nof_layers, Nref, g.nof_ch_symbols)
        tbs.append(tb)
        cfgs.append(srsgpu.PdschTransportBlock(seg.base_graph, rv, g.qm, g.nof_layers, g.nof_ch_symbols, Nref))
        want.append(cw)
    got = srsgpu.PdschEncoder(ctx).encode_batch(tbs, cfgs)
    for i, (a, b) in enumerate(zip(got, want)):
        assert np.array_equal(a, b), (i, cfgs[i])


def test_pdsch_encoder_slot_100mhz(ctx):
    """The benchmark slot (64 UEs, 4 layers, 256QAM MCS 27) against the oracle."""
    import srsgpu
    from srsgpu import sch
    orc = Oracle()
    rng = np.random.default_rng(8)
    tbs, cfgs, want = [], [], []
    for g in sch.slot_100mhz_4x4():
        seg = g.segmentation()
        tb = rng.integers(0, 256, seg.tbs // 8).astype(np.uint8)
        cw, _, _ = oracle_pdsch_encode(orc, tb, seg.base_graph, 0, g.qm, g.nof_layers, 0, g.nof_ch_symbols)
        tbs.append(tb)
        cfgs.append(srsgpu.PdschTransportBlock(seg.base_graph, 0, g.qm, g.nof_layers, g.nof_ch_symbols))
        want.append(cw)
    got = srsgpu.PdschEncoder(ctx).encode_batch(tbs, cfgs)
    for a, b in zip(got, want):
        assert np.array_equal(a, b)


def test_pdsch_encoder_packed_kernel_every_lifting_size(ctx):
    """The packed kernel (Z % 32 == 0) against the oracle and against the byte kernel (SRSGPU_OPTION_ENCODER_BYTE_KERNEL)
    on grants covering every (BG, Z) with Z a multiple of 32 that the TBS tables reach, every Qm and rv."""
    import os
    import srsgpu
    from srsgpu import sch
    orc = Oracle()
    rng = np.random.default_rng(32)
    tables = list(sch.MCS_TABLE_256QAM.values())
    seen, tbs, cfgs, want = set(), [], [], []
    for _ in range(4000):
        qm, r = tables[int(rng.integers(0, len(tables)))]
        g = sch.UeGrant(int(rng.integers(1, 140)), int(rng.integers(1, 5)), qm, r,
                        nof_symb_sh=int(rng.integers(2, 15)))
        seg = g.segmentation()
        key = (seg.base_graph, seg.lifting_size, g.qm)
        if seg.lifting_size % 32 or key in seen or seg.tbs > 200000:
            continue
        seen.add(key)
        rv = int(rng.integers(0, 4))
        tb = rng.integers(0, 256, seg.tbs // 8).astype(np.uint8)
        cw, _, _ = oracle_pdsch_encode(orc, tb, seg.base_graph, rv, g.qm, g.nof_layers, 0, g.nof_ch_symbols)
        tbs.append(tb)
        cfgs.append(srsgpu.PdschTransportBlock(seg.base_graph, rv, g.qm, g.nof_layers, g.nof_ch_symbols))
        want.append(cw)
    assert len({(b, z) for b, z, _ in seen}) >= 12, sorted(seen)
    got = srsgpu.PdschEncoder(ctx).encode_batch(tbs, cfgs)
    for i, (a, b) in enumerate(zip(got, want)):
        assert np.array_equal(a, b), (i, cfgs[i])
    with ctx.options(encoder_byte_kernel=1):
        byte = srsgpu.PdschEncoder(ctx).encode_batch(tbs, cfgs)
    for a, b in zip(got, byte):
        assert np.array_equal(a, b)


def test_crc_table_arena_long_running_cell(ctx):
    """A long-running cell with link adaptation (advisor round 1): 60 PDSCH encoder + PUSCH decoder plans, each TB of
    a distinct large size (its optional per-length TB CRC table is up to 1.2 M words of the 16 M-word arena), created
    and destroyed, then 12 kept alive at once; plans needing new codeblock CRC lengths are still created (required
    tables evict unreferenced cached ones, optional ones always leave a reserve) and still encode correctly."""
    import srsgpu
    from srsgpu import sch
    orc = Oracle()

    def nsym(nb):
        return ((nb * 8 * 10 // 8 + 7) // 8 + 3) // 4 * 4  # G / Qm at code rate ~0.8, a multiple of the layers

    for i in range(60):
        nb = 150000 + 97 * i
        arr, _, _, _ = srsgpu.make_pdsch_configs([nb], [srsgpu.PdschTransportBlock(1, 0, 8, 4, nsym(nb))])
        srsgpu.PdschEncoderPlan(ctx, arr).close()
        seg = sch.segment(nb * 8, 1, 8, 4, nsym(nb))
        ul = srsgpu.PuschTransportBlock(nb, 1, 0, 8, 4, nsym(nb), new_data=True)
        arr, *_ = srsgpu.make_pusch_tb_configs([ul], [seg.nof_segments],
                                               [66 * seg.codeblocks[0].lifting_size])
        srsgpu.PuschDecoderPlan(ctx, srsgpu.IMPL_SIMD, arr).close()
    live = []
    for i in range(12):
        nb = 140000 + 89 * i
        arr, _, _, _ = srsgpu.make_pdsch_configs([nb], [srsgpu.PdschTransportBlock(1, 0, 8, 4, nsym(nb))])
        live.append(srsgpu.PdschEncoderPlan(ctx, arr))
    rng = np.random.default_rng(3)
    tbs, cfgs, want = [], [], []
    for nb in (3007, 20013, 61005):  # new codeblock lengths
        tb = rng.integers(0, 256, nb).astype(np.uint8)
        cw, _, _ = oracle_pdsch_encode(orc, tb, 1, 0, 8, 4, 0, nsym(nb))
        tbs.append(tb)
        cfgs.append(srsgpu.PdschTransportBlock(1, 0, 8, 4, nsym(nb)))
        want.append(cw)
    got = srsgpu.PdschEncoder(ctx).encode_batch(tbs, cfgs)
    for a, b in zip(got, want):
        assert np.array_equal(a, b)
    for p in live:
        p.close()


def test_pdsch_encoder_aligned_plan_without_memset(ctx):
    """A plan whose codeblocks all cover whole 32-bit words (4 layers of 256QAM) and whose codewords tile the output
    skips the output memset (capi.cpp: zero_output): on an output pre-filled with 0xAB (encode_batch) it must give the
    oracle's codewords, as the memset path (SRSGPU_OPTION_ENCODER_ZERO_OUTPUT) does; a 1-layer QPSK TB in the plan brings the
    memset back (edge words ORed)."""
    import srsgpu
    from srsgpu import sch
    orc = Oracle()
    rng = np.random.default_rng(11)
    grants = list(sch.slot_100mhz_4x4())[:8]
    tbs, cfgs, want = [], [], []
    qm2, r2 = [v for v in sch.MCS_TABLE_256QAM.values() if v[0] == 2][0]
    for g in grants + [sch.UeGrant(3, 1, qm2, r2, nof_symb_sh=11)]:
        seg = g.segmentation()
        tb = rng.integers(0, 256, seg.tbs // 8).astype(np.uint8)
        cw, _, _ = oracle_pdsch_encode(orc, tb, seg.base_graph, 0, g.qm, g.nof_layers, 0, g.nof_ch_symbols)
        tbs.append(tb)
        cfgs.append(srsgpu.PdschTransportBlock(seg.base_graph, 0, g.qm, g.nof_layers, g.nof_ch_symbols))
        want.append(cw)
    enc = srsgpu.PdschEncoder(ctx)
    for zero in (0, 1):
        with ctx.options(encoder_zero_output=zero):
            for n in (len(grants), len(grants) + 1):  # aligned plan; plus the unaligned TB
                got = enc.encode_batch(tbs[:n], cfgs[:n])
                for i, (a, b) in enumerate(zip(got, want[:n])):
                    assert np.array_equal(a, b), (zero, n, i)
