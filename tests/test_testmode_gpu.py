"""configs[4]: the du_low test mode's traffic on the GPU - one test UE owning all 273 PRB in every slot (max TBS,
MCS 27, 4 DL layers), continuous slots of the du_high default TDD pattern DDDDDDSUUU (du_high_config.h:503-511; the
special slot carries an 8-symbol PDSCH with DM-RS in symbols 2 and 7), the whole period captured once as a HIP graph
and replayed slot period after slot period with fresh data:

* DL: every replay draws new TB payloads on the GPU inside the graph (srsgpu.slot.DownlinkGroup, fresh_tbs). Each
  period's codewords, grids and samples must equal an eager run of the same plans on the drawn payloads, and a
  loopback receiver (the GPU's own OFDM demodulator -> 4-layer estimator -> MMSE demodulator -> decoder, after AWGN)
  must decode every drawn TB of the period;
* UL: the period's 3 UL slots (one max-TBS single-layer PUSCH each, ZF, the reference-runnable profile) rotate over
  independently synthesised UE transmissions; every replay must decode that transmission's TBs.
"""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def ctx():
    import srsgpu
    return srsgpu.Context(0)


def test_testmode_cells_follow_the_tdd_pattern():
    from srsgpu import slot as slotlib
    dl, sp, ul = slotlib.tdd_testmode_cells(2)
    assert [dl.slot_index(s) for s in range(dl.nof_slots)] == [0, 1, 2, 3, 4, 5, 10, 11, 12, 13, 14, 15]
    assert [sp.slot_index(s) for s in range(sp.nof_slots)] == [6, 16]
    assert [ul.slot_index(s) for s in range(ul.nof_slots)] == [7, 8, 9, 17, 18, 19]
    assert sp.nof_symbols == 8 and sp.dmrs_mask == (1 << 2) | (1 << 7)
    # Max TBS of 273 PRB, 256QAM MCS 27 (TS 38.214 5.1.3.2): 4 layers x 12 data symbols, 4 layers x 6, 1 layer x 12.
    assert [c.segs[0].tbs for c in (dl, sp, ul)] == [1179864, 590128, 295176]


@pytest.mark.gpu
def test_testmode_continuous_periods_with_fresh_payloads(ctx):
    import torch
    import srsgpu
    from srsgpu import slot as slotlib
    dl_cell, sp_cell, ul_cell = slotlib.tdd_testmode_cells(1, dl_layers=4, ul_layers=1)
    dls = [slotlib.DownlinkPipeline(ctx, c) for c in (dl_cell, sp_cell)]
    tbs = [torch.zeros(d.tb_total, dtype=torch.uint8, device="cuda") for d in dls]
    group = slotlib.DownlinkGroup(dls, tbs, fresh_tbs=True)
    ul = slotlib.UplinkPipeline(ctx, ul_cell, equalizer=srsgpu.EQ_ZF)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(21)
    ul_sets = []
    for k in range(2):  # two different UE transmissions of the period's UL slots
        sent = torch.randint(0, 256, (sum(ul.tb_bytes),), generator=gen, device="cuda", dtype=torch.uint8)
        x = slotlib.synthesize_uplink(ctx, ul_cell, sent, snr_db=30.0, seed=40 + k, cfo_hz_max=300.0)
        ul_sets.append((sent, x))
    samples = torch.zeros_like(ul_sets[0][1])
    # Loopback receivers for the DL slots (the GPU transmitter's own output, identity channel + AWGN).
    rx = [slotlib.UplinkPipeline(ctx, c) for c in (dl_cell, sp_cell)]
    eager = [slotlib.DownlinkPipeline(ctx, c) for c in (dl_cell, sp_cell)]
    eager_group = slotlib.DownlinkGroup(eager, tbs, fresh_tbs=False)

    s_dl, s_ul = torch.cuda.Stream(), torch.cuda.Stream()

    def period():
        cur = torch.cuda.current_stream()
        s_dl.wait_stream(cur)
        s_ul.wait_stream(cur)
        group.execute(s_dl)
        ul.execute(samples, s_ul)
        cur.wait_stream(s_dl)
        cur.wait_stream(s_ul)

    period()  # warm-up (plans' first launches) outside the capture
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        period()
    stream = torch.cuda.current_stream()
    prev = None
    for step in range(4):
        sent, x = ul_sets[step % 2]
        samples.copy_(x)
        graph.replay()
        torch.cuda.synchronize()
        drawn = [t.clone() for t in tbs]
        if prev is not None:  # fresh payloads on every replay
            for a, b in zip(drawn, prev):
                assert not torch.equal(a, b)
        prev = drawn
        # The graph's DL outputs equal an eager run of identical plans on the same payloads.
        eager_group.execute(stream)
        torch.cuda.synchronize()
        for d, e in zip(dls, eager):
            assert torch.equal(d.d_cw, e.d_cw)
            assert torch.equal(d.d_grid, e.d_grid)
            assert torch.equal(d.d_samples, e.d_samples)
        # Loopback: every DL TB of the period decodes to the drawn payload.
        for d, r, t in zip(dls, rx, drawn):
            y = d.d_samples
            rms = float(y.square().mean().sqrt())
            noisy = y + torch.randn(y.shape, generator=gen, device="cuda") * (rms * 10 ** (-35 / 20))
            r.execute(noisy, stream)
            torch.cuda.synchronize()
            ok = r.d_tb_ok.cpu().numpy()
            assert ok.all(), (step, np.nonzero(ok == 0)[0])
            assert torch.equal(r.d_tbs, t)
        # UL: this period's UE transmission.
        ok = ul.d_tb_ok.cpu().numpy()
        assert ok.all(), (step, np.nonzero(ok == 0)[0])
        assert torch.equal(ul.d_tbs, sent)


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["full", "special"])
def test_testmode_dl_max_tbs_codeword_and_grid_vs_oracle(ctx, which):
    """configs[4]'s DL at its real size against the oracle: the 1 179 864-bit max-TBS TB of a full DL slot (4 layers,
    DM-RS 2 + 11; 140 codeblocks) and the 590 128-bit TB of the special slot's 8-symbol PDSCH (DM-RS 2 + 7), each
    encoded by the GPU PDSCH encoder (bit-exact vs the oracle's TB CRC -> segmentation -> CB CRC -> LDPC -> rate
    matching) and mapped with its DM-RS into the slot's 4-port grid (bit-exact vs the oracle modulator + DM-RS
    restatements, both pinned against the reference)."""
    import torch
    import pdsch_dmrs_oracle as M
    from chain_lib import oracle_pdsch_encode
    from oracle_lib import Oracle
    from srsgpu import slot as slotlib
    orc = Oracle()
    dl_cell, sp_cell, _ = slotlib.tdd_testmode_cells(1)
    cell = dl_cell if which == "full" else sp_cell
    pipe = slotlib.DownlinkPipeline(ctx, cell)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(7)
    d_tbs = torch.randint(0, 256, (pipe.tb_total,), generator=gen, device="cuda", dtype=torch.uint8)
    pipe.execute(d_tbs, torch.cuda.current_stream())
    torch.cuda.synchronize()
    u, seg = cell.ues[0], cell.segs[0]
    tb = d_tbs[: seg.tbs // 8].cpu().numpy()
    want_cw, _, _ = oracle_pdsch_encode(orc, tb, seg.base_graph, 0, u.qm, u.nof_layers, 0, u.nof_ch_symbols)
    cw_bytes = pipe.d_cw.cpu().numpy()
    got_cw = np.unpackbits(cw_bytes[pipe.cw_offsets[0]: pipe.cw_offsets[0] + (seg.cw_length + 7) // 8])[: seg.cw_length]
    assert np.array_equal(got_cw, want_cw)
    # Slot 0 grid: the oracle modulator (identity precoding, 4 layers on 4 ports) over the DM-RS oracle's grid.
    w = np.eye(4, dtype=np.complex64)
    dm = dict(slot=cell.slot_index(0), scrambling_id=500, n_scid=0, dmrs_type2=0, nof_layers=4, nof_ports=4,
              dmrs_symbol_mask=cell.dmrs_mask, reference_point_k_rb=0, rb_start=0, nof_rb=273,
              amplitude=slotlib.DMRS_BETA)
    want = M.dmrs_map(dm, w, 273)
    mod = dict(rnti=0x4601, n_id=500, qm=u.qm, nof_layers=4, nof_ports=4, bwp_start_rb=0, bwp_size_rb=273, rb_start=0,
               nof_rb=273, start_symbol=0, nof_symbols=cell.nof_symbols, dmrs_symbol_mask=cell.dmrs_mask,
               dmrs_type2=0, nof_cdm_groups_without_data=2, scaling=1.0)
    want = orc.pdsch_modulate(mod, w, np.packbits(want_cw), seg.cw_length, 273, grid=want)
    got = pipe.d_grid.cpu().numpy().view(np.uint16).reshape(cell.nof_slots, 4, 14, 12 * 273, 2)[0]
    assert np.array_equal(got, want)
