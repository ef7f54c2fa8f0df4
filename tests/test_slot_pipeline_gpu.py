"""End-to-end slot pipelines on the GPU (srsgpu.slot): the bench's 100 MHz 4x4 64-UE slot, 2 slots.

UL: UE transmitter (GPU encoder / DM-RS / modulator) -> random unitary 4x4 channel + AWGN (35 dB) -> OFDM modulation
-> receive chain (OFDM demodulation, channel estimation, MMSE demodulation, PUSCH decoding): every TB must pass its CRC
and equal what was sent. DL: encoder -> DM-RS -> modulator -> OFDM modulator; the OFDM-demodulated samples must give
back the DL grid (bf16 round trip), and the grid's PDSCH REs must equal the PDSCH modulator's output."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import srsgpu
    return srsgpu.Context(0)


def test_uplink_pipeline_decodes_every_tb(ctx):
    import torch
    from srsgpu import sch
    from srsgpu import slot as slotlib
    ues = sch.slot_100mhz_4x4()
    segs = [u.segmentation() for u in ues]
    cell = slotlib.CellSlots(ues, segs, 2)
    ul = slotlib.UplinkPipeline(ctx, cell)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(5)
    tbs = torch.randint(0, 256, (sum(ul.tb_bytes),), generator=gen, device="cuda", dtype=torch.uint8)
    samples = slotlib.synthesize_uplink(ctx, cell, tbs, snr_db=35.0, seed=3)
    stream = torch.cuda.current_stream()
    ul.execute(samples, stream)
    torch.cuda.synchronize()
    ok = ul.d_tb_ok.cpu().numpy()
    assert ok.all(), np.nonzero(ok == 0)[0]
    assert np.array_equal(ul.d_tbs.cpu().numpy(), tbs.cpu().numpy())
    nv = ul.d_nv.cpu().numpy().reshape(-1, 4)
    # 35 dB SNR on unit-power layers: the estimated noise (AWGN plus the estimator's residual) stays well below 25 dB.
    assert np.all(nv > 0) and np.all(nv < 10 ** (-25 / 10))


def test_downlink_pipeline_round_trip(ctx):
    import torch
    import srsgpu
    from srsgpu import sch
    from srsgpu import slot as slotlib
    ues = sch.slot_100mhz_4x4()
    segs = [u.segmentation() for u in ues]
    cell = slotlib.CellSlots(ues, segs, 2)
    dl = slotlib.DownlinkPipeline(ctx, cell)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(6)
    tbs = torch.randint(0, 256, (dl.tb_total,), generator=gen, device="cuda", dtype=torch.uint8)
    stream = torch.cuda.current_stream()
    dl.execute(tbs, stream)
    back = torch.zeros_like(dl.d_grid)
    demod = srsgpu.OfdmPlan(ctx, False, slotlib.NUMEROLOGY, cell.grid_prb, slotlib.DFT_SIZE,
                            1.0 / (slotlib.TX_SCALE * slotlib.DFT_SIZE), slotlib.CENTER_FREQ_HZ, [0, 1], 4)
    demod.execute(dl.d_samples, back)
    torch.cuda.synchronize()
    from ofdm_cases import bf16_close
    a = dl.d_grid.cpu().numpy().view(np.uint16).reshape(-1, 2)
    b = back.cpu().numpy().view(np.uint16).reshape(-1, 2)
    ok, frac = bf16_close(b, a)
    assert ok and frac < 0.05, frac
    # Every RE of the 2 slots is written: PDSCH on 13 symbols, DM-RS on symbol 2 where, with identity precoding, port p
    # carries the DM-RS of layer p only, so half of each port's symbol-2 REs (the other CDM group) are exactly zero
    # (+0 or -0: a zero weight times a negative DM-RS value is -0).
    zero = ~np.any((a & 0x7fff) != 0, axis=1)
    assert abs(np.mean(zero) - 1 / 28) < 1e-3, np.mean(zero)


def test_uplink_compact_estimates_match_per_symbol_layout(ctx):
    """The compact channel-estimate layout (one row per allocation) gives LLRs identical to the reference's
    per-symbol layout, and its row equals every symbol row of the per-symbol estimate."""
    import torch
    import srsgpu
    from srsgpu import sch
    from srsgpu import slot as slotlib
    ues = sch.slot_100mhz_4x4()
    segs = [u.segmentation() for u in ues]
    cell = slotlib.CellSlots(ues, segs, 1)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(7)
    tbs = torch.randint(0, 256, (sum(u.segmentation().tbs // 8 for u in ues),), generator=gen, device="cuda",
                        dtype=torch.uint8)
    samples = slotlib.synthesize_uplink(ctx, cell, tbs, snr_db=30.0, seed=4)
    stream = torch.cuda.current_stream()
    full = slotlib.UplinkPipeline(ctx, cell, estimate_layout=srsgpu.CE_PER_SYMBOL)
    compact = slotlib.UplinkPipeline(ctx, cell, estimate_layout=srsgpu.CE_COMPACT)
    full.execute(samples, stream)
    compact.execute(samples, stream)
    torch.cuda.synchronize()
    assert np.array_equal(full.d_llrs.cpu().numpy(), compact.d_llrs.cpu().numpy())
    assert np.array_equal(full.d_nv.cpu().numpy(), compact.d_nv.cpu().numpy())
    ce_full = full.d_ce.cpu().numpy().reshape(4, cell.nof_ports, 14, cell.nsc)
    ce_comp = compact.d_ce.cpu().numpy().reshape(4, cell.nof_ports, 14, cell.nsc)
    for l in range(14):
        assert np.array_equal(ce_full[:, :, l], ce_comp[:, :, 0])
    assert compact.d_tb_ok.cpu().numpy().all()


def test_pipelines_replay_as_hip_graph(ctx):
    """The DL and UL plans are allocation-free and capture-safe: both legs captured once into one HIP graph (forked
    onto two streams) and replayed give the same codewords, grids, samples, LLRs and decoded TBs as eager launches."""
    import torch
    from srsgpu import sch
    from srsgpu import slot as slotlib
    ues = sch.slot_100mhz_4x4()
    segs = [u.segmentation() for u in ues]
    cell = slotlib.CellSlots(ues, segs, 2)
    dl = slotlib.DownlinkPipeline(ctx, cell)
    ul = slotlib.UplinkPipeline(ctx, cell)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(9)
    dl_tbs = torch.randint(0, 256, (dl.tb_total,), generator=gen, device="cuda", dtype=torch.uint8)
    ul_tbs = torch.randint(0, 256, (dl.tb_total,), generator=gen, device="cuda", dtype=torch.uint8)
    samples = slotlib.synthesize_uplink(ctx, cell, ul_tbs, snr_db=35.0, seed=11)
    s_dl, s_ul = torch.cuda.Stream(), torch.cuda.Stream()

    def pipeline():
        cur = torch.cuda.current_stream()
        s_dl.wait_stream(cur)
        s_ul.wait_stream(cur)
        dl.execute(dl_tbs, s_dl)
        ul.execute(samples, s_ul)
        cur.wait_stream(s_dl)
        cur.wait_stream(s_ul)

    pipeline()
    torch.cuda.synchronize()
    outs = [dl.d_cw, dl.d_grid, dl.d_samples, ul.d_llrs, ul.d_tbs, ul.d_tb_ok, ul.d_iters]
    eager = [t.clone() for t in outs]
    for t in outs:
        t.zero_()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        pipeline()
    for t in outs:  # capture does not execute: clear again and replay twice
        t.zero_()
    graph.replay()
    graph.replay()
    torch.cuda.synchronize()
    for a, b in zip(eager, outs):
        assert torch.equal(a, b)
    assert ul.d_tb_ok.cpu().numpy().all()
    assert torch.equal(ul.d_tbs, ul_tbs)
