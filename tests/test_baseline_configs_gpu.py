"""BASELINE.json's single-GPU configurations as end-to-end parity cases (the bench runs configs[3]'s 100 MHz 4x4 slot).

configs[1] "PDSCH processor n78 20 MHz SISO 64-QAM, single slot": the DL pipeline (PDSCH encoder -> DM-RS ->
modulator, srsgpu.slot.DownlinkPipeline) on a 51-PRB one-port grid, compared stage by stage with the oracle
composition (codeword and grid bit-exact), then the 20 MHz OFDM modulator (1024-point DFT) against the complex128
oracle within 2e-5 x RMS.

configs[2] "PUSCH processor n78 100 MHz 2x2 256-QAM with DM-RS channel est + MMSE equalizer": the UL pipeline (OFDM
demodulator -> DM-RS estimator -> demodulator -> decoder) on a full 273-PRB two-port slot of 2-layer 256QAM UEs,
received through a random unitary 2x2 channel at 35 dB: every TB decodes to the bytes sent, with the MMSE equaliser
(multi-layer: an extension, parity unpinned) and the reference's ZF 2xN equaliser (pinned)."""
import numpy as np
import pytest

from chain_lib import oracle_pdsch_encode
from oracle_lib import Oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import srsgpu
    return srsgpu.Context(0)


def test_config1_pdsch_20mhz_siso_64qam(ctx):
    import torch
    import pdsch_dmrs_oracle as D
    import ofdm_oracle as O
    import srsgpu
    from ofdm_cases import rel_err
    from srsgpu import sch
    from srsgpu import slot as slotlib
    prb = 51
    ue = sch.UeGrant(prb, 1, 6, 719.0)
    seg = ue.segmentation()
    cell = slotlib.CellSlots([ue], [seg], 1, grid_prb=prb, nof_ports=1)
    dl = slotlib.DownlinkPipeline(ctx, cell)
    rng = np.random.default_rng(20)
    tb = rng.integers(0, 256, seg.tbs // 8).astype(np.uint8)
    dl.execute(torch.from_numpy(tb).cuda(), torch.cuda.current_stream())
    torch.cuda.synchronize()

    orc = Oracle()
    cw, _, _ = oracle_pdsch_encode(orc, tb, seg.base_graph, 0, ue.qm, 1, 0, ue.nof_ch_symbols)
    got_cw = np.unpackbits(dl.d_cw.cpu().numpy())[: cw.size]
    assert np.array_equal(got_cw, cw)

    w = np.ones((1, 1), np.complex64)
    mcfg = dict(rnti=0x4601, n_id=500, qm=6, nof_layers=1, nof_ports=1, bwp_start_rb=0, bwp_size_rb=prb, rb_start=0,
                nof_rb=prb, start_symbol=0, nof_symbols=14, dmrs_symbol_mask=1 << slotlib.DMRS_SYMBOL, dmrs_type2=0,
                nof_cdm_groups_without_data=2, scaling=1.0)
    want = orc.pdsch_modulate(mcfg, w, np.packbits(cw), cw.size, prb)
    dcfg = dict(slot=0, scrambling_id=500, n_scid=0, dmrs_type2=0, nof_layers=1, nof_ports=1,
                dmrs_symbol_mask=1 << slotlib.DMRS_SYMBOL, reference_point_k_rb=0, rb_start=0, nof_rb=prb,
                amplitude=slotlib.DMRS_BETA)
    want[:, slotlib.DMRS_SYMBOL] = D.dmrs_map(dcfg, w, prb)[:, slotlib.DMRS_SYMBOL]
    grid = dl.d_grid.cpu().numpy().view(np.uint16).reshape(1, 14, 12 * prb, 2)
    assert np.array_equal(grid, want)

    scale, fc = 1.0 / 32, 3.5e9
    samples = srsgpu.OfdmSlotModulator(ctx, 1, prb, 1024, scale, fc).modulate(grid, 0)
    assert rel_err(samples, O.modulate(want, 1, prb, 1024, False, scale, fc, 0)) < 2e-5


@pytest.mark.parametrize("equalizer", ["mmse", "zf"])
def test_config2_pusch_100mhz_2x2_256qam(ctx, equalizer):
    import torch
    import srsgpu
    from srsgpu import sch
    from srsgpu import slot as slotlib
    ues = [sch.UeGrant(17 if i < 15 else 18, 2, 8, 797.0) for i in range(16)]  # 273 PRB
    assert sum(u.n_prb for u in ues) == 273
    segs = [u.segmentation() for u in ues]
    cell = slotlib.CellSlots(ues, segs, 1, nof_ports=2)
    eq = srsgpu.EQ_MMSE if equalizer == "mmse" else srsgpu.EQ_ZF
    ul = slotlib.UplinkPipeline(ctx, cell, equalizer=eq)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(22)
    tbs = torch.randint(0, 256, (sum(ul.tb_bytes),), generator=gen, device="cuda", dtype=torch.uint8)
    samples = slotlib.synthesize_uplink(ctx, cell, tbs, snr_db=35.0, seed=23)
    ul.execute(samples, torch.cuda.current_stream())
    torch.cuda.synchronize()
    ok = ul.d_tb_ok.cpu().numpy()
    assert ok.all(), np.nonzero(ok == 0)[0]
    assert torch.equal(ul.d_tbs, tbs)
