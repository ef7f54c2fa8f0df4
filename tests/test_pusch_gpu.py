"""GPU parity of the PUSCH codeblock path (rate dematching + HARQ combining + LDPC decoding + CB CRC) against the
oracle composition (tests/chain_lib.py), through the C ABI (srsgpu_pusch_cb_plan_*)."""
import numpy as np
import pytest

from chain_lib import bits_to_llrs, crc_for_tb, oracle_pdsch_encode, oracle_pusch_cb_decode
from oracle_lib import BG_K, BG_N_SHORT, Oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def orc():
    return Oracle()


@pytest.fixture(scope="module")
def ctx():
    import srsgpu
    return srsgpu.Context(0)


@pytest.mark.parametrize("dec_type,mode", [("avx2", 1), ("generic", 0)])
def test_rate_dematch_random_configs(orc, ctx, dec_type, mode):
    """HARQ buffer after the plan == oracle rate dematcher, 300 random codeblocks in one batch (random rv, Qm, LBRM,
    fillers, lengths ending inside / after the first pass, copy and combine, +/-127 inputs)."""
    import srsgpu
    rng = np.random.default_rng(31 + mode)
    cbs, llrs, inits = [], [], []
    while len(cbs) < 300:
        bg = int(rng.integers(1, 3))
        Z = int(rng.choice([2, 3, 5, 16, 24, 64, 144, 384]))
        N = BG_N_SHORT[bg] * Z
        nsys = (BG_K[bg] - 2) * Z
        qm = int(rng.choice([1, 2, 4, 6, 8]))
        F = int(rng.integers(0, nsys // 3 + 1))
        Nref = int(rng.choice([0, int(N * rng.uniform(0.75, 0.99))]))
        if 0 < Nref <= nsys:
            continue
        E = qm * int(rng.integers(1, 3 * N // qm))
        cbs.append(srsgpu.PuschCodeblock(bg, Z, int(rng.integers(0, 4)), qm, E, nof_filler_bits=F, Nref=Nref,
                                         new_data=bool(rng.integers(0, 2)), max_iterations=1))
        llrs.append(rng.integers(-127, 128, E).astype(np.int8))
        inits.append(rng.integers(-127, 128, N).astype(np.int8))
    dec = srsgpu.PuschCodeblockDecoder(ctx, dec_type)
    _, harq, _ = dec.decode(llrs, cbs, harq=np.concatenate(inits))
    off = 0
    for c, llr, init in zip(cbs, llrs, inits):
        N = BG_N_SHORT[c.base_graph] * c.lifting_size
        want = orc.rate_dematch(mode, c.base_graph, c.lifting_size, c.rv, c.modulation_order, c.Nref,
                                c.nof_filler_bits, int(c.new_data), llr, init)
        assert np.array_equal(harq[off:off + N], want), c
        off += N


def _ue_codeblocks(srsgpu, seg, rv, qm, new_data, early_stop, max_iter=8):
    return [srsgpu.PuschCodeblock(seg.base_graph, seg.lifting_size, rv, qm, cb.rm_length,
                                  nof_filler_bits=cb.nof_filler_bits, crc_poly=crc_for_tb(seg),
                                  nof_crc_bits=cb.nof_crc_bits, new_data=new_data, use_early_stop=early_stop,
                                  max_iterations=max_iter) for cb in seg.codeblocks]


@pytest.mark.parametrize("early_stop", [True, False])
def test_pusch_chain_with_harq_retransmission(orc, ctx, early_stop):
    """Transport blocks of several grants: encode (oracle), noisy LLRs, rv0 first transmission, then an rv2
    retransmission combined in the device HARQ buffer; every step equals the oracle chain (iterations, bits, HARQ
    buffer, CRC flags)."""
    import srsgpu
    from srsgpu import sch
    rng = np.random.default_rng(77 + early_stop)
    dec = srsgpu.PuschCodeblockDecoder(ctx, "avx2")
    grants = [sch.UeGrant(4, 4, 8, 948), sch.UeGrant(5, 2, 6, 772), sch.UeGrant(12, 1, 4, 434),
              sch.UeGrant(2, 1, 2, 120), sch.UeGrant(30, 2, 8, 682.5)]
    all_cbs, all_llrs, oracle_state = [], [], []
    tx = {}
    for gi, g in enumerate(grants):
        seg = g.segmentation()
        tb = rng.integers(0, 256, seg.tbs // 8).astype(np.uint8)
        tx[gi] = (tb, seg)
    for rv, new_data, noise in ((0, True, 9.0), (2, False, 9.0)):
        cbs, llrs = [], []
        for gi, g in enumerate(grants):
            tb, seg = tx[gi]
            cw, seg, _ = oracle_pdsch_encode(orc, tb, seg.base_graph, rv, g.qm, g.nof_layers, 0, g.nof_ch_symbols)
            llr = bits_to_llrs(rng, cw, amp=6.0, noise=noise)
            cbs += _ue_codeblocks(srsgpu, seg, rv, g.qm, new_data, early_stop)
            for cb in seg.codeblocks:
                llrs.append(llr[cb.cw_offset: cb.cw_offset + cb.rm_length])
        if new_data:
            harq_g = None
            crc_g = None
            oracle_state = [(np.zeros(BG_N_SHORT[c.base_graph] * c.lifting_size, np.int8), False) for c in cbs]
        res, harq_g, crc_g = dec.decode(llrs, cbs, harq=harq_g, cb_crc_ok=crc_g)
        off = 0
        new_state = []
        n_ok = 0
        for i, (c, llr) in enumerate(zip(cbs, llrs)):
            h, ok = oracle_state[i]
            r, bits, h2, ok2 = oracle_pusch_cb_decode(orc, 1, c, llr, h, ok)
            N = BG_N_SHORT[c.base_graph] * c.lifting_size
            assert np.array_equal(harq_g[off:off + N], h2), (rv, i)
            off += N
            r_g, bits_g = res[i]
            assert (r_g if r_g is not None else -1) == r, (rv, i)
            if bits is not None:
                assert np.array_equal(bits_g, bits), (rv, i)
            assert bool(crc_g[i]) == ok2
            n_ok += ok2
            new_state.append((h2, ok2))
        oracle_state = new_state
    assert n_ok > 0


def test_pusch_decoder_tb_level(orc, ctx):
    """TB-level PUSCH decoder (segmentation, CB decoding, concatenation, TB CRC24A) for 60 transport blocks of random
    grants at several SNRs, then an rv2 retransmission: TB CRC flags, recovered TBs and per-CB iteration counts equal
    the oracle composition of pusch_decoder_impl."""
    import srsgpu
    from srsgpu import sch
    rng = np.random.default_rng(5)
    dec = srsgpu.PuschDecoder(ctx, "avx2")
    tables = list(sch.MCS_TABLE_256QAM.values())
    grants, tbs = [], []
    while len(grants) < 60:
        qm, r = tables[int(rng.integers(0, len(tables)))]
        g = sch.UeGrant(int(rng.integers(1, 40)), int(rng.integers(1, 5)), qm, r, nof_symb_sh=int(rng.integers(6, 15)))
        seg = g.segmentation()
        grants.append((g, seg))
        tbs.append(rng.integers(0, 256, seg.tbs // 8).astype(np.uint8))
    state = {}
    for rv, new_data in ((0, True), (2, False)):
        llrs, cfgs = [], []
        for i, ((g, seg), tb) in enumerate(zip(grants, tbs)):
            cw, _, _ = oracle_pdsch_encode(orc, tb, seg.base_graph, rv, g.qm, g.nof_layers, 0, g.nof_ch_symbols)
            noise = [2.0, 6.0, 9.0, 12.0][i % 4]
            llrs.append(bits_to_llrs(rng, cw, amp=6.0, noise=noise))
            cfgs.append(srsgpu.PuschTransportBlock(seg.tbs // 8, seg.base_graph, rv, g.qm, g.nof_layers,
                                                   g.nof_ch_symbols, new_data=new_data, nof_ldpc_iterations=6))
        ok, got_tbs, iters = dec.decode_batch(llrs, cfgs)
        n_ok = 0
        for i, ((g, seg), tb, llr) in enumerate(zip(grants, tbs, llrs)):
            cbs = _ue_codeblocks(srsgpu, seg, rv, g.qm, new_data, True, max_iter=6)
            st = state.get(i) or [(np.zeros(BG_N_SHORT[c.base_graph] * c.lifting_size, np.int8), False, None)
                                  for c in cbs]
            new_st, want_iters = [], []
            for c, cb, (h, flag, msg) in zip(cbs, seg.codeblocks, st):
                if new_data:
                    flag = False
                r, bits, h2, ok2 = oracle_pusch_cb_decode(orc, 1, c, llr[cb.cw_offset: cb.cw_offset + cb.rm_length],
                                                          h, flag)
                want_iters.append(r)
                new_st.append((h2, ok2, bits if bits is not None else msg))
            assert iters[i] == want_iters, (rv, i)
            all_ok = all(x[1] for x in new_st)
            if seg.nof_segments == 1:
                tb_ok = new_st[0][1]
            elif all_ok:
                tb_ok = True  # every CB CRC passed; a TB CRC mismatch would reset the flags (not expected here)
            else:
                tb_ok = False
            assert ok[i] == tb_ok, (rv, i)
            if tb_ok:
                assert np.array_equal(got_tbs[i], tb), (rv, i)
                n_ok += 1
            state[i] = new_st
        assert n_ok >= 10


def test_pusch_decoder_large_unaligned_tbs(orc, ctx):
    """A byte-aligned TBS outside the TS 38.214 tables, large enough that the codeblock index of a TB bit needs the
    corrected magic division (526 344 bits: C = 63 codeblocks of 8 356 data bits, not byte-aligned, TB bit index x
    codeblock bits >= 2^32): clean LLRs decode to the sent bytes with the TB CRC passing."""
    import srsgpu
    from srsgpu import sch
    rng = np.random.default_rng(9)
    tbs_bits = 526344
    qm, layers, nsym = 8, 4, 73200  # G = 585 600 bits (code rate 0.9)
    seg = sch.segment(tbs_bits, 1, qm, layers, nsym)
    assert seg.nof_segments == 63 and (tbs_bits + 24) % (8 * 63) != 0
    tb = rng.integers(0, 256, tbs_bits // 8).astype(np.uint8)
    cw, _, _ = oracle_pdsch_encode(orc, tb, 1, 0, qm, layers, 0, nsym)
    llr = bits_to_llrs(rng, cw, amp=10.0, noise=0.0)
    dec = srsgpu.PuschDecoder(ctx, "avx2")
    ok, got, iters = dec.decode_batch([llr], [srsgpu.PuschTransportBlock(tbs_bits // 8, 1, 0, qm, layers, nsym,
                                                                         new_data=True, nof_ldpc_iterations=6)])
    assert len(iters[0]) == 63 and ok[0], (len(iters[0]), ok[0])
    assert np.array_equal(got[0], tb)


@pytest.mark.parametrize("dec_type,mode", [("avx2", 1), ("generic", 0)])
def test_fused_rate_dematch_in_decoder(orc, ctx, dec_type, mode):
    """First transmissions that are a plain copy (rv 0, no LBRM, ninfo <= E <= V, even Z) are dematched inside the
    packed decoder (DEC_FLAG_FUSED_DM): 160 such codeblocks mixed with 40 that keep the separate rate dematcher, over a
    HARQ buffer of random old content; iterations, bits, HARQ buffer and CRC flags equal the oracle composition and the
    unfused plan (SRSGPU_OPTION_DECODER_FUSED_DEMATCH = 0)."""
    import srsgpu
    rng = np.random.default_rng(404 + mode)
    cbs, llrs, inits = [], [], []
    while len(cbs) < 200:
        fusable = len(cbs) < 160
        bg = int(rng.integers(1, 3))
        Z = int(rng.choice([2, 4, 16, 36, 64, 112, 144, 208, 288, 384] if fusable else [3, 5, 64, 384]))
        N = BG_N_SHORT[bg] * Z
        nsys = (BG_K[bg] - 2) * Z
        qm = int(rng.choice([1, 2, 4, 6, 8]))
        F = int(rng.integers(0, nsys // 3 + 1))
        ninfo = nsys - F
        if fusable:
            lo, hi = -(-ninfo // qm), (N - F) // qm
            if lo > hi:
                continue
            E, rv, Nref = qm * int(rng.integers(lo, hi + 1)), 0, 0
        else:
            E, rv, Nref = qm * int(rng.integers(1, 2 * N // qm)), int(rng.integers(0, 4)), 0
        cbs.append(srsgpu.PuschCodeblock(bg, Z, rv, qm, E, nof_filler_bits=F, Nref=Nref, new_data=True,
                                         use_early_stop=bool(rng.integers(0, 2)), max_iterations=4))
        # Mostly a noisy all-zero codeword (decodes, CRC passes), a quarter pure noise (fails).
        amp = 0.0 if rng.random() < 0.25 else 10.0
        llrs.append(np.clip(np.round(amp + 4.0 * rng.standard_normal(E)), -127, 127).astype(np.int8))
        inits.append(rng.integers(-127, 128, N).astype(np.int8))
    init = np.concatenate(inits)
    dec = srsgpu.PuschCodeblockDecoder(ctx, dec_type)
    res_f, harq_f, crc_f = dec.decode(llrs, cbs, harq=init.copy())
    with ctx.options(decoder_fused_dematch=0):
        res_u, harq_u, crc_u = dec.decode(llrs, cbs, harq=init.copy())
    assert np.array_equal(harq_f, harq_u)
    assert np.array_equal(np.asarray(crc_f), np.asarray(crc_u))
    off, n_ok = 0, 0
    for i, (c, llr, h0) in enumerate(zip(cbs, llrs, inits)):
        r, bits, h2, ok2 = oracle_pusch_cb_decode(orc, mode, c, llr, h0, False)
        N = BG_N_SHORT[c.base_graph] * c.lifting_size
        assert np.array_equal(harq_f[off:off + N], h2), (i, c)
        off += N
        for res in (res_f, res_u):
            r_g, bits_g = res[i]
            assert (r_g if r_g is not None else -1) == r, (i, c)
            if bits is not None:
                assert np.array_equal(bits_g, bits), (i, c)
        assert bool(crc_f[i]) == ok2, (i, c)
        n_ok += ok2
    assert 30 <= n_ok < 200


def test_codeblock_sharded_decode_assemble(orc, ctx):
    """Codeblock-sharded decoding on the device (srsgpu/dist.py CodeblockShard's data path, three ranks emulated on one
    GPU): every rank's codeblock range decoded by a srsgpu_pusch_cb_plan from its LLR span into its own HARQ buffers,
    the messages / flags placed in slot-wide buffers, the TBs joined by srsgpu_pusch_decoder_plan_assemble. TB bytes,
    TB and CB CRC flags and messages equal the TB-level plan decoding everything, for a 63-codeblock TB (configs[4]'s
    shape) plus smaller TBs, one of them too noisy to decode."""
    import torch

    import srsgpu
    from srsgpu import dist as sdist
    from srsgpu import sch
    rng = np.random.default_rng(17)
    g1, g2 = sch.UeGrant(30, 2, 8, 682.5), sch.UeGrant(12, 1, 6, 600.0)
    grants = [(sch.segment(526344, 1, 8, 4, 73200), 8, 4, 73200, 0.0),
              (g1.segmentation(), g1.qm, g1.nof_layers, g1.nof_ch_symbols, 5.0),
              (g2.segmentation(), g2.qm, g2.nof_layers, g2.nof_ch_symbols, 40.0)]
    tbs_cfg, segs, tbs, llrs = [], [], [], []
    for seg, qm, layers, nsym, noise in grants:
        tbs_bits = seg.tbs
        tb = rng.integers(0, 256, tbs_bits // 8).astype(np.uint8)
        cw, _, _ = oracle_pdsch_encode(orc, tb, seg.base_graph, 0, qm, layers, 0, nsym)
        llrs.append(bits_to_llrs(rng, cw, amp=10.0, noise=noise))
        tbs_cfg.append(srsgpu.PuschTransportBlock(tbs_bits // 8, seg.base_graph, 0, qm, layers, nsym, new_data=True,
                                                  nof_ldpc_iterations=6))
        segs.append(seg)
        tbs.append(tb)
    nof_cbs = [s.nof_segments for s in segs]
    arr, nllr, nharq, ncb, ntb = srsgpu.make_pusch_tb_configs(
        tbs_cfg, nof_cbs, [BG_N_SHORT[s.base_graph] * s.lifting_size for s in segs])
    dev = torch.device("cuda", 0)
    d_llrs = torch.from_numpy(np.concatenate(llrs)).to(dev)
    plan = srsgpu.PuschDecoderPlan(ctx, srsgpu.IMPL_BY_NAME["avx2"], arr)

    # Reference: the TB-level plan decodes every codeblock.
    ref = dict(crc=torch.zeros(ncb, dtype=torch.uint8, device=dev),
               msgs=torch.zeros(ncb * sdist.CB_MSG_STRIDE, dtype=torch.uint8, device=dev),
               tbs=torch.zeros(ntb, dtype=torch.uint8, device=dev), ok=torch.zeros(len(segs), dtype=torch.uint8,
                                                                                   device=dev))
    plan.execute(d_llrs, torch.zeros(nharq, dtype=torch.int8, device=dev), ref["crc"], ref["msgs"],
                 torch.zeros(ncb, dtype=torch.int32, device=dev), ref["tbs"], ref["ok"])

    # Sharded: the slot's codeblocks in order, each with its codeword LLR range.
    flat, cb_llr = [], []
    for i, seg in enumerate(segs):
        for cb in seg.codeblocks:
            flat.append(srsgpu.PuschCodeblock(seg.base_graph, seg.lifting_size, 0, tbs_cfg[i].modulation_order,
                                              cb.rm_length, nof_filler_bits=cb.nof_filler_bits,
                                              crc_poly=crc_for_tb(seg), nof_crc_bits=cb.nof_crc_bits,
                                              max_iterations=6))
            cb_llr.append((arr[i].llr_offset + cb.cw_offset, cb.rm_length))
    world = 3
    all_crc = torch.zeros(ncb, dtype=torch.uint8, device=dev)
    all_msgs = torch.zeros(ncb * sdist.CB_MSG_STRIDE, dtype=torch.uint8, device=dev)
    for r in range(world):
        rg = sdist.shard_range(len(flat), world, r)
        b0 = cb_llr[rg.start][0]
        span = d_llrs[b0: cb_llr[rg.stop - 1][0] + cb_llr[rg.stop - 1][1]].clone()  # what scatter_llrs hands rank r
        cfg, lo, ho, _ = srsgpu.make_pusch_cb_configs([flat[i] for i in rg])
        for j, i in enumerate(rg):
            assert cfg[j].llr_offset == cb_llr[i][0] - b0  # contiguous codeblocks: the packed offsets are the span's
            cfg[j].out_offset = j * sdist.CB_MSG_STRIDE
        msgs = torch.zeros(len(rg) * sdist.CB_MSG_STRIDE, dtype=torch.uint8, device=dev)
        crc = torch.zeros(len(rg), dtype=torch.uint8, device=dev)
        cbp = srsgpu.PuschCbPlan(ctx, srsgpu.IMPL_BY_NAME["avx2"], cfg)
        cbp.execute(span, torch.zeros(ho, dtype=torch.int8, device=dev), msgs,
                    torch.zeros(len(rg), dtype=torch.int32, device=dev), crc)
        torch.cuda.synchronize(dev)
        cbp.close()
        all_msgs[rg.start * sdist.CB_MSG_STRIDE: rg.stop * sdist.CB_MSG_STRIDE].copy_(msgs)  # what gather does
        all_crc[rg.start: rg.stop].copy_(crc)
    got_tbs = torch.zeros(ntb, dtype=torch.uint8, device=dev)
    got_ok = torch.zeros(len(segs), dtype=torch.uint8, device=dev)
    plan.assemble(all_crc, all_msgs, got_tbs, got_ok)
    torch.cuda.synchronize(dev)
    plan.close()
    assert got_ok.tolist() == ref["ok"].tolist() == [1, 1, 0], (got_ok.tolist(), ref["ok"].tolist())
    assert torch.equal(all_crc, ref["crc"])
    assert torch.equal(got_tbs, ref["tbs"])
    ok_cbs = ref["crc"].cpu().numpy().astype(bool)
    m_got = all_msgs.view(ncb, -1).cpu().numpy()[ok_cbs]
    m_ref = ref["msgs"].view(ncb, -1).cpu().numpy()[ok_cbs]
    assert np.array_equal(m_got, m_ref)
    off = 0
    for seg, tb, good in zip(segs, tbs, [1, 1, 0]):
        if good:
            assert np.array_equal(got_tbs[off: off + tb.size].cpu().numpy(), tb)
        off += tb.size


def test_pusch_decoder_sliced_tb_stage(orc, ctx):
    """Plans whose TBs are all segmented, byte-aligned and one above 16 KB run the TB stage over 4 KB slices (several
    workgroups per TB, the last finisher checks the CRC): clean TBs decode to the sent bytes, a TB with a failed
    codeblock is flagged, and - through srsgpu_pusch_decoder_plan_assemble on a corrupted message with its codeblock
    flag still set - a TB CRC mismatch clears every codeblock flag of that TB only. Executed twice (the slice counters
    and sums reset themselves)."""
    import torch

    import srsgpu
    from srsgpu import sch
    rng = np.random.default_rng(23)
    grants = [(sch.UeGrant(273, 1, 8, 948), 0.0), (sch.UeGrant(100, 2, 8, 800), 0.0), (sch.UeGrant(60, 1, 8, 900), 60.0)]
    cfgs, segs, tbs, llrs = [], [], [], []
    for g, noise in grants:
        seg = g.segmentation()
        assert seg.nof_segments > 1
        tb = rng.integers(0, 256, seg.tbs // 8).astype(np.uint8)
        cw, _, _ = oracle_pdsch_encode(orc, tb, seg.base_graph, 0, g.qm, g.nof_layers, 0, g.nof_ch_symbols)
        llrs.append(bits_to_llrs(rng, cw, amp=10.0, noise=noise))
        cfgs.append(srsgpu.PuschTransportBlock(seg.tbs // 8, seg.base_graph, 0, g.qm, g.nof_layers, g.nof_ch_symbols,
                                               new_data=True, nof_ldpc_iterations=6))
        segs.append(seg)
        tbs.append(tb)
    assert max(t.size for t in tbs) > 16384
    arr, nllr, nharq, ncb, ntb = srsgpu.make_pusch_tb_configs(
        cfgs, [s.nof_segments for s in segs], [BG_N_SHORT[s.base_graph] * s.lifting_size for s in segs])
    dev = torch.device("cuda", 0)
    d_llrs = torch.from_numpy(np.concatenate(llrs)).to(dev)
    plan = srsgpu.PuschDecoderPlan(ctx, srsgpu.IMPL_BY_NAME["avx2"], arr)
    for _ in range(2):
        crc = torch.zeros(ncb, dtype=torch.uint8, device=dev)
        msgs = torch.zeros(ncb * srsgpu.CB_MSG_STRIDE, dtype=torch.uint8, device=dev)
        out = torch.zeros(ntb, dtype=torch.uint8, device=dev)
        ok = torch.zeros(len(segs), dtype=torch.uint8, device=dev)
        plan.execute(d_llrs, torch.zeros(nharq, dtype=torch.int8, device=dev), crc, msgs,
                     torch.zeros(ncb, dtype=torch.int32, device=dev), out, ok)
        torch.cuda.synchronize(dev)
        assert ok.tolist() == [1, 1, 0], ok.tolist()
        off = 0
        for tb, good in zip(tbs, [1, 1, 0]):
            if good:
                assert np.array_equal(out[off: off + tb.size].cpu().numpy(), tb)
            off += tb.size
    # TB CRC mismatch: flip one data byte of TB 1's second codeblock message (its CB flag stays set).
    c1 = segs[0].nof_segments + 1
    msgs[c1 * srsgpu.CB_MSG_STRIDE + 5] ^= 0x10
    ok2 = torch.zeros(len(segs), dtype=torch.uint8, device=dev)
    plan.assemble(crc, msgs, out, ok2)
    torch.cuda.synchronize(dev)
    plan.close()
    assert ok2.tolist() == [1, 0, 0], ok2.tolist()
    flags = crc.cpu().numpy()
    n0, n1 = segs[0].nof_segments, segs[1].nof_segments
    assert flags[:n0].all() and not flags[n0:n0 + n1].any()


def test_copy_spans():
    """srsgpu_copy_spans (the slot batches' rx-grid gather): several spans of different sizes in one launch, each
    destination equal to its source, the bytes around them untouched; unaligned sizes refused."""
    import torch
    import srsgpu
    srsgpu.Context(0)
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(5)
    srcs = [torch.randint(0, 255, (n,), dtype=torch.uint8, generator=g).to(dev) for n in (16, 4096, 733824, 48)]
    big = torch.full((sum(x.numel() for x in srcs) + 64 * len(srcs),), 7, dtype=torch.uint8, device=dev)
    dsts, off = [], 0
    for x in srcs:
        dsts.append(big[off:off + x.numel()])
        off += x.numel() + 64
    keep = srsgpu.copy_spans(list(zip(srcs, dsts)))
    torch.cuda.synchronize()
    del keep
    off = 0
    for x, d in zip(srcs, dsts):
        assert torch.equal(x, d)
        gap = big[off + x.numel():off + x.numel() + 64]
        assert int(gap.min()) == 7 == int(gap.max())
        off += x.numel() + 64
    with pytest.raises(srsgpu.SrsGpuError):
        srsgpu.copy_spans([(srcs[0][:8], dsts[0][:8])])


def test_merge_spans():
    """srsgpu_merge_spans (the multi-device PDSCH batch's gather): every destination word whose source word is not the
    sentinel takes the source's, the others keep their value; vectors of four sentinel words, of none and mixed ones."""
    import torch
    import srsgpu
    srsgpu.Context(0)
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(9)
    n = 3276 * 4
    src = torch.randint(0, 2 ** 31 - 1, (3, n), dtype=torch.int64, generator=g).to(torch.int32)
    sentinel = -1  # 0xffffffff
    src[0, : n // 2] = sentinel                          # whole vectors of sentinels
    src[1, torch.randperm(n, generator=g)[: n // 3]] = sentinel  # mixed vectors
    dst = torch.randint(0, 2 ** 31 - 1, (3, n), dtype=torch.int64, generator=g).to(torch.int32)
    want = torch.where(src != sentinel, src, dst)
    s_d, d_d = src.to(dev), dst.to(dev)
    keep = srsgpu.merge_spans([(s_d[i], d_d[i]) for i in range(3)])
    torch.cuda.synchronize()
    del keep
    assert torch.equal(d_d.cpu(), want)


def test_pusch_decoder_harq_in_arena(orc, ctx):
    """srsgpu_pusch_decoder_plan_execute_arena (each codeblock's HARQ soft buffer in a slot of a scattered, garbage-
    initialised arena, addressed through a per-codeblock pointer table) equals srsgpu_pusch_decoder_plan_execute over a
    contiguous batch HARQ buffer bit for bit, for a new transmission (fused and separate rate dematching, odd and even
    lifting sizes) and an rv2 retransmission that combines with the soft bits left in the arena: codeblock CRC flags,
    messages and iteration counts, TBs, TB CRC flags and every HARQ soft bit."""
    import torch
    import srsgpu
    from srsgpu import sch
    rng = np.random.default_rng(11)
    dev = torch.device("cuda", 0)
    tables = list(sch.MCS_TABLE_256QAM.values())
    grants, tbs = [], []
    while len(grants) < 40:
        qm, r = tables[int(rng.integers(0, len(tables)))]
        g = sch.UeGrant(int(rng.integers(1, 40)), int(rng.integers(1, 5)), qm, r, nof_symb_sh=int(rng.integers(6, 15)))
        seg = g.segmentation()
        grants.append((g, seg))
        tbs.append(rng.integers(0, 256, seg.tbs // 8).astype(np.uint8))
    nof_cbs = [seg.nof_segments for _, seg in grants]
    cb_len = [BG_N_SHORT[seg.base_graph] * seg.lifting_size for _, seg in grants]
    slot_bytes = 66 * 384
    ncb = sum(nof_cbs)
    arena = torch.from_numpy(rng.integers(-128, 128, 2 * ncb * slot_bytes).astype(np.int8)).to(dev)
    perm = rng.permutation(2 * ncb)[:ncb]
    ptrs = torch.tensor([arena.data_ptr() + int(p) * slot_bytes for p in perm], dtype=torch.int64, device=dev)
    state = None
    for rv, new_data in ((0, True), (2, False)):
        llrs, cfgs = [], []
        for i, ((g, seg), tb) in enumerate(zip(grants, tbs)):
            cw, _, _ = oracle_pdsch_encode(orc, tb, seg.base_graph, rv, g.qm, g.nof_layers, 0, g.nof_ch_symbols)
            llrs.append(bits_to_llrs(rng, cw, amp=6.0, noise=[2.0, 6.0, 9.0, 12.0][i % 4]))
            cfgs.append(srsgpu.PuschTransportBlock(seg.tbs // 8, seg.base_graph, rv, g.qm, g.nof_layers,
                                                   g.nof_ch_symbols, new_data=new_data, nof_ldpc_iterations=6))
        arr, nllr, nharq, ncb2, ntb = srsgpu.make_pusch_tb_configs(cfgs, nof_cbs, cb_len)
        assert ncb2 == ncb
        if state is None:
            state = [dict(harq=torch.zeros(nharq, dtype=torch.int8, device=dev)) for _ in range(2)]
            for st in state:
                st["crc"] = torch.zeros(ncb, dtype=torch.uint8, device=dev)
                st["msgs"] = torch.zeros(ncb * srsgpu.CB_MSG_STRIDE, dtype=torch.uint8, device=dev)
        d_llrs = torch.from_numpy(np.concatenate(llrs).astype(np.int8)).to(dev)
        assert d_llrs.numel() == nllr
        plan = srsgpu.PuschDecoderPlan(ctx, srsgpu.IMPL_BY_NAME["avx2"], arr)
        outs = []
        for k, st in enumerate(state):
            it = torch.zeros(ncb, dtype=torch.int32, device=dev)
            tb_out = torch.zeros(max(ntb, 1), dtype=torch.uint8, device=dev)
            tb_ok = torch.zeros(len(cfgs), dtype=torch.uint8, device=dev)
            if k == 0:
                plan.execute(d_llrs, st["harq"], st["crc"], st["msgs"], it, tb_out, tb_ok)
            else:
                plan.execute_arena(d_llrs, ptrs, st["crc"], st["msgs"], it, tb_out, tb_ok)
            outs.append((it, tb_out, tb_ok))
        torch.cuda.synchronize(dev)
        plan.close()
        for a, b in zip(outs[0], outs[1]):
            assert torch.equal(a, b), rv
        assert torch.equal(state[0]["crc"], state[1]["crc"]), rv
        assert torch.equal(state[0]["msgs"], state[1]["msgs"]), rv
        harq = state[0]["harq"].cpu().numpy()
        arena_h = arena.cpu().numpy()
        c = 0
        for t in range(len(cfgs)):
            for i in range(nof_cbs[t]):
                off = int(arr[t].harq_offset) + i * cb_len[t]
                slot = int(perm[c]) * slot_bytes
                assert np.array_equal(harq[off: off + cb_len[t]], arena_h[slot: slot + cb_len[t]]), (rv, t, i)
                c += 1
        assert int(outs[0][2].sum()) >= 8


def test_pusch_decoder_two_codeblock_workgroups(orc, ctx):
    """Two codeblocks of Z = 144 .. 192 per workgroup (SRSGPU_OPTION_DECODER_PAIRS: ldpc_decode_pairs_kernel,
    fused rate dematching on first transmissions, the separate dematcher for the rv2 retransmission) equal the
    one-codeblock kernel (the default) bit for bit: TB flags, TBs, per-CB iteration counts and the HARQ soft bits, over an odd
    number of such codeblocks (a workgroup with an empty slot) mixed with other lifting sizes; and the oracle."""
    import torch
    import srsgpu
    from srsgpu import sch
    rng = np.random.default_rng(23)
    grants, tbs = [], []
    # 4-5 PRB 256QAM grants (Z = 192 / 224, the bench's UL), Z = 144 / 160 / 176 grants and a 12-PRB one (Z = 384).
    while len(grants) < 41:
        k = len(grants) % 6
        nprb, qm, rate, ns = [(4, 8, 948.0, 12), (5, 8, 948.0, 12), (2, 8, 682.5, 12), (4, 8, 948.0, 10),
                              (3, 8, 682.5, 10), (12, 4, 616.0, 12)][k]
        g = sch.UeGrant(nprb, 1, qm, rate, nof_symb_sh=ns)
        seg = g.segmentation()
        grants.append((g, seg))
        tbs.append(rng.integers(0, 256, seg.tbs // 8).astype(np.uint8))
    zs = {seg.lifting_size for _, seg in grants}
    assert {144, 160, 176, 192} <= zs, zs
    results = {}
    for pk2 in ("1", "0"):
        with ctx.options(decoder_pairs=int(pk2)):
            dec = srsgpu.PuschDecoder(ctx, "avx2")
            out = []
            for rv, new_data in ((0, True), (2, False)):
                llrs, cfgs = [], []
                for i, ((g, seg), tb) in enumerate(zip(grants, tbs)):
                    cw, _, _ = oracle_pdsch_encode(orc, tb, seg.base_graph, rv, g.qm, g.nof_layers, 0, g.nof_ch_symbols)
                    r = np.random.default_rng(1000 * rv + i)
                    llrs.append(bits_to_llrs(r, cw, amp=8.0, noise=[1.0, 3.0, 7.0][i % 3]))
                    cfgs.append(srsgpu.PuschTransportBlock(seg.tbs // 8, seg.base_graph, rv, g.qm, g.nof_layers,
                                                           g.nof_ch_symbols, new_data=new_data, nof_ldpc_iterations=6))
                ok, got, iters = dec.decode_batch(llrs, cfgs)
                out.append((ok, [t.copy() for t in got], iters, dec.harq[0].cpu().numpy().copy()))
                print(f"PK2={pk2} rv{rv}: TBs ok {sum(ok)}/{len(ok)}, iterations {sorted({x for v in iters for x in v})}")
            results[pk2] = out
    for a, b in zip(results["1"], results["0"]):
        assert a[0] == b[0]
        assert all(np.array_equal(x, y) for x, y in zip(a[1], b[1]))
        assert a[2] == b[2]
        assert np.array_equal(a[3], b[3])
    # The one-codeblock kernel against the oracle for the first transmission (as test_pusch_decoder_tb_level).
    ok0, got0, iters0, _ = results["0"][0]
    n_ok = 0
    for i, ((g, seg), tb) in enumerate(zip(grants, tbs)):
        if ok0[i]:
            assert np.array_equal(got0[i], tb), i
            n_ok += 1
    assert n_ok >= 10
