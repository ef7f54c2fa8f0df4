"""Upper-PHY slot processors on the GPU (row b6): the reference's OWN uplink_processor_impl and
downlink_processor_single_executor_impl (compiled from its sources by oracle/build_chain.sh) run once over the
reference's CPU channel processors and once over the GPU slot batches of integration/upper_phy_gpu.cpp, which gather
a slot's PUSCH / PDSCH PDUs into one launch sequence (tests/chain_harness.py: UpperPhy). Row b8: every GPU processor
here is obtained only through the GPU factories' create() (uplink_processor_factory / downlink_processor_factory of
integration/upper_phy_factories_gpu.cpp, with the GPU pusch_processor_factory / pdsch_processor_factory for the PDUs
the batches do not cover), as upper_phy_factories.cpp obtains its processors; their create_pdu_validator() equals the
reference's validators.

  * UL: multi-UE slots (different sizes, modulations, CFOs, delays, SNRs, one UE over the DC subcarrier, one with
    HARQ-ACK on PUSCH, whose UL-SCH stream the batch demultiplexes on the GPU) registered in the reference's PDU repository;
    handle_rx_symbol(13). Then a second slot with retransmissions (rv 2, new_data = false) of the first slot's failed
    TBs combined with the soft bits the batch kept in HBM (arena slots = the rx buffer pool's absolute codeblock
    identifiers), plus new UEs. Equal per (RNTI, HARQ id): TB CRC, payload, number of codeblocks; within the
    tolerances of tests/test_chain_gpu.py (the GPU LLRs equal the reference's or differ by one quantisation step):
    LDPC mean iterations +-0.5, SINR 0.1 dB, EVM 2e-3, TA 2 Tc, CFO 0.05 Hz, EPRE / RSRP 0.01 dB.
  * DL: a slot of PDSCHs (1-4 layers on 4 ports, random precoding, 64 / 256QAM) into a grid that already holds other
    channels' content: the grid the reference's processor sends is bit-exact with the CPU processors' one.
"""
import numpy as np
import pytest

from ofdm_oracle import bf16_to_complex
from pusch_demod_cases import bf16
from srsgpu import sch

pytestmark = pytest.mark.gpu

T_C = 1.0 / (480000 * 4096)
P = 4


@pytest.fixture(scope="module", params=["sync", "async", "multi3_copy", "multi3_copy_async", "multi1_rccl"])
def procs(request):
    """The reference's CPU processors and the GPU batches, the latter completing synchronously (the PUSCH task returns
    with the results notified), asynchronously (results notified from the GPU service's completion thread), or as the
    multi-GPU batch of row b7 (and its DL counterpart, the PDSCH slot batch over the same three shards): the slot's UEs
    sharded by RNTI over the device list {0, 0, 0} (three shards with their
    own launch plans, HARQ arenas and grid copies on one GPU, results gathered by peer copies; synchronous, or
    asynchronous with the replay on the batch's completion thread) or over {0} with the RCCL transport (world size 1:
    the gather is an ncclSend / ncclRecv pair in one group). Every mode must equal the reference's CPU processors,
    hence the single-device batch."""
    import chain_harness as H
    cpu = H.UpperPhy(0, H.UL_CPU, P)
    extra = {"sync": 0, "async": H.UL_ASYNC, "multi3_copy": H.UL_MULTI_COPY,
             "multi3_copy_async": H.UL_MULTI_COPY | H.UL_ASYNC, "multi1_rccl": H.UL_MULTI_RCCL}
    gpu = H.UpperPhy(0, H.UL_GPU_BATCH | extra[request.param], P)
    gpu.mode = request.param
    yield cpu, gpu
    cpu.close()
    gpu.close()


def grant(p):
    nd = bin(p.dmrs_mask).count("1")
    return sch.UeGrant(p.nof_rb, p.nof_layers, p.qm, p.target_code_rate, nof_symb_sh=p.nof_symbols,
                       nof_dmrs_symbols=nd)


def received_grid(rng, chain, ues, tbs, snr_db):
    """Every UE's transmission (the reference's transmitter, chain_ue_tx) through its own random flat channel per rx
    port, delay and CFO, summed, plus AWGN: (P, 14, nsc, 2) bf16."""
    import pusch_chest_oracle as C
    nsc = 12 * 273
    y = np.zeros((P, 14, nsc), np.complex128)
    k = np.arange(nsc)
    ep = C.symbol_start_epochs(1)
    for (p, cfo, delay, gain_db), tb in zip(ues, tbs):
        x = bf16_to_complex(chain.ue_tx(p, tb))
        g = (rng.normal(size=(P, p.nof_layers)) + 1j * rng.normal(size=(P, p.nof_layers))) / np.sqrt(2 * p.nof_layers)
        g *= 10 ** (gain_db / 20)
        ramp = np.exp(-2j * np.pi * k * delay / 4096)
        yu = np.einsum("pl,lsk->psk", g, x) * ramp[None, None, :]
        yu *= np.exp(2j * np.pi * cfo / 30000.0 * ep)[None, :, None]
        y += yu
    nv = 10 ** (-snr_db / 10)
    y += (rng.normal(size=y.shape) + 1j * rng.normal(size=y.shape)) * np.sqrt(nv / 2)
    return bf16(y)


def check_equal(ref, got, what):
    assert len(ref) == len(got), what
    rk = {(d["rnti"], d["harq_id"]): (d, tb) for d, tb in ref}
    gk = {(d["rnti"], d["harq_id"]): (d, tb) for d, tb in got}
    assert rk.keys() == gk.keys(), what
    for key, (r, tbr) in rk.items():
        g, tbg = gk[key]
        w = (what, key)
        assert g["tb_crc_ok"] == r["tb_crc_ok"], (w, r, g)
        assert g["nof_cbs"] == r["nof_cbs"], w
        if r["tb_crc_ok"]:
            assert np.array_equal(tbg, tbr), w
        if r["ldpc_obs"] > 0:
            assert abs(g["ldpc_mean"] - r["ldpc_mean"]) <= 0.5, (w, r["ldpc_mean"], g["ldpc_mean"])
        assert abs(g["sinr_db"] - r["sinr_db"]) < 0.1, (w, r["sinr_db"], g["sinr_db"])
        assert abs(g["evm"] - r["evm"]) < 2e-3, (w, r["evm"], g["evm"])
        assert abs(g["ta_s"] - r["ta_s"]) <= 2 * T_C, (w, r["ta_s"], g["ta_s"])
        if not np.isnan(r["cfo_hz"]):
            assert abs(g["cfo_hz"] - r["cfo_hz"]) < 0.05, (w, r["cfo_hz"], g["cfo_hz"])
        assert abs(g["epre_db"] - r["epre_db"]) < 0.01 and abs(g["rsrp_db"] - r["rsrp_db"]) < 0.01, (w, r, g)
        assert (g["harq_ack_status"], g["harq_ack_bits"]) == (r["harq_ack_status"], r["harq_ack_bits"]), (w, r, g)
        for f in ("csi1_status", "csi1_size", "csi1_bits", "csi2_status", "csi2_size", "csi2_bits"):
            assert g[f] == r[f], (w, f, r, g)


def ul_ues(rng, H, start_rnti, n, harq0, low_snr=()):
    """n UEs side by side from RB 0: (params, CFO Hz, delay samples, gain dB)."""
    out, rb = [], 0
    for i in range(n):
        nrb = int(rng.choice([4, 5, 8, 12, 17]))
        qm, rate = [(8, 948.0), (6, 772.0), (4, 616.0), (2, 308.0)][i % 4]
        p = H.params(rnti=start_rnti + i, harq_id=harq0 + i, nof_rb=nrb, rb_start=rb, qm=qm, target_code_rate=rate,
                     nof_ports=P)
        rb += nrb
        gain = -22.0 if i in low_snr else 0.0
        out.append((p, float(rng.uniform(-250, 250)), float(rng.uniform(-3, 3)), gain))
    return out, rb


def test_uplink_processor_gpu_batch_equals_reference(procs):
    import chain_harness as H
    cpu, gpu = procs
    chain = H.Chain(0)
    try:
        rng = np.random.default_rng(2024)
        ues, rb = ul_ues(rng, H, 0x4601, 14, 0, low_snr=(4, 9))
        # A UE over the DC subcarrier (its estimate is zeroed there) and one with HARQ-ACK on PUSCH.
        dc = H.params(rnti=0x4700, harq_id=20, nof_rb=10, rb_start=rb, qm=6, target_code_rate=772.0, nof_ports=P,
                      dc_position=12 * (rb + 4) + 6)
        ack = H.params(rnti=0x4701, harq_id=21, nof_rb=8, rb_start=rb + 10, qm=4, target_code_rate=616.0, nof_ports=P,
                       nof_harq_ack=2)
        ues += [(dc, 50.0, 1.0, 0.0), (ack, -90.0, 0.0, 0.0)]
        tbs, sizes = [], []
        for p, *_ in ues:
            seg = grant(p).segmentation()
            p.base_graph = seg.base_graph
            tbs.append(rng.integers(0, 256, seg.tbs // 8).astype(np.uint8))
            sizes.append(seg.tbs // 8)
        grid = received_grid(rng, chain, ues, tbs, 28.0)
        pdus = [p for p, *_ in ues]
        ref = cpu.ul_slot(7, pdus, sizes, grid)
        before = gpu.multi_transfer_counters()
        got = gpu.ul_slot(7, pdus, sizes, grid)
        after = gpu.multi_transfer_counters()
        check_equal(ref, got, "slot 7")
        if gpu.mode.startswith("multi3"):
            # One host-to-device grid transfer for the slot whatever the number of devices; the two other shards
            # receive only their UEs' subcarrier bands from the root's copy (less than the whole grid each).
            assert after["host_uploads"] - before["host_uploads"] == 1, (before, after)
            assert after["shard_copies"] - before["shard_copies"] == 2, (before, after)
            moved = after["shard_bytes"] - before["shard_bytes"]
            assert 0 < moved < 2 * P * 14 * 12 * 273 * 4, moved
        ok = {d["rnti"]: d["tb_crc_ok"] for d, _ in ref}
        ack_res = next(d for d, _ in got if d["rnti"] == ack.rnti)
        assert ack_res["harq_ack_status"] >= 0, ack_res  # the HARQ-ACK field was reported
        data_ok = [ok[p.rnti] for p, *_ in ues if p.nof_harq_ack == 0]
        assert sum(data_ok) == len(data_ok) - 2, ok  # every UE decodes but the two faded ones
        for (p, *_), tb in zip(ues, tbs):
            if ok[p.rnti] and p.nof_harq_ack == 0:
                got_tb = next(t for d, t in got if d["rnti"] == p.rnti)
                assert np.array_equal(got_tb[: tb.size], tb)

        # Slot 8: the failed TBs again as rv 2 (combined with the kept soft bits) next to new UEs.
        retx = [(u, tb) for u, tb in zip(ues, tbs) if not ok[u[0].rnti] and u[0].nof_harq_ack == 0]
        ues2, tbs2 = [], []
        rb = 0
        for (p, cfo, delay, gain), tb in retx:
            q = H.params(**{f: getattr(p, f) for f, _ in H.ChainParams._fields_})
            q.rv, q.new_data, q.rb_start, q.slot = 2, 0, rb, 8
            rb += q.nof_rb
            ues2.append((q, cfo, delay, 0.0))
            tbs2.append(tb)
        new, _ = ul_ues(rng, H, 0x4800, 6, 40)
        for p, cfo, delay, gain in new:
            p.rb_start += rb
            p.slot = 8  # the UE's DM-RS and scrambling of slot 8 (the processor's slot)
            seg = grant(p).segmentation()
            p.base_graph = seg.base_graph
            ues2.append((p, cfo, delay, gain))
            tbs2.append(rng.integers(0, 256, seg.tbs // 8).astype(np.uint8))
        grid2 = received_grid(rng, chain, ues2, tbs2, 28.0)
        pdus2 = [p for p, *_ in ues2]
        sizes2 = [t.size for t in tbs2]
        ref2 = cpu.ul_slot(8, pdus2, sizes2, grid2)
        got2 = gpu.ul_slot(8, pdus2, sizes2, grid2)
        check_equal(ref2, got2, "slot 8")
        ok2 = {d["rnti"]: d["tb_crc_ok"] for d, _ in ref2}
        # The 64QAM retransmission decodes after combining; the 256QAM rate-0.93 one does not (rv 2 carries almost no
        # systematic bits and its first transmission was faded) - on the reference as on the GPU (check_equal above).
        assert sum(ok2[p.rnti] for (p, *_), _ in retx) >= 1, ok2
    finally:
        chain.close()


def test_uplink_processor_gpu_batch_csi_part2_equals_reference(procs):
    """UCI with CSI Part 2 on PUSCH (pusch_processor_impl.cpp:55-101): the UL-SCH bit count depends on the decoded CSI
    Part 1, so the batch decodes the UL-SCH of such a PDU in a second launch from the replay, after the reference's UCI
    decoder has decoded CSI Part 1 and its feedback has set CSI Part 2 - placed from the symbol completing CSI Part 1
    on (ulsch_demultiplex_impl.cpp:241). Fixed-size and CSI-Part-1-dependent CSI Part 2 sizes, with and without
    HARQ-ACK, next to plain UEs; results (TB, CRC, LDPC statistics, HARQ-ACK, CSI Part 1 and Part 2 status, size and
    bits, CSI) equal the reference's CPU processors."""
    import chain_harness as H
    cpu, gpu = procs
    chain = H.Chain(0)
    try:
        rng = np.random.default_rng(606)
        ues, rb = ul_ues(rng, H, 0x4901, 4, 30)
        specs = [dict(nof_csi_part1=4, csi2_size0=20), dict(nof_csi_part1=7, csi2_size0=12, csi2_size1=30),
                 dict(nof_harq_ack=3, nof_csi_part1=11, csi2_size0=8), dict(nof_csi_part1=2, csi2_size0=3),
                 dict(nof_harq_ack=1, nof_csi_part1=20, csi2_size0=40, csi2_size1=5)]
        for i, sp in enumerate(specs):
            nrb = [12, 16, 10, 8, 20][i]
            p = H.params(rnti=0x4a00 + i, harq_id=40 + i, nof_rb=nrb, rb_start=rb, qm=[4, 6, 2, 4, 6][i],
                         target_code_rate=[616.0, 772.0, 308.0, 616.0, 772.0][i], nof_ports=P, **sp)
            rb += nrb
            ues.append((p, float(rng.uniform(-200, 200)), 0.0, 0.0))
        tbs, sizes = [], []
        for p, *_ in ues:
            seg = grant(p).segmentation()
            p.base_graph = seg.base_graph
            tbs.append(rng.integers(0, 256, seg.tbs // 8).astype(np.uint8))
            sizes.append(seg.tbs // 8)
        grid = received_grid(rng, chain, ues, tbs, 28.0)
        pdus = [p for p, *_ in ues]
        ref = cpu.ul_slot(9, pdus, sizes, grid)
        got = gpu.ul_slot(9, pdus, sizes, grid)
        check_equal(ref, got, "slot 9, CSI Part 2")
        csi2 = [d for d, _ in ref if d["rnti"] >= 0x4a00]
        assert all(d["csi1_status"] >= 0 for d in csi2), csi2
        # CSI Part 2 reported whenever CSI Part 1 decoded (the path through the second launch was taken).
        assert any(d["csi2_status"] >= 0 for d in csi2), csi2
    finally:
        chain.close()


def test_downlink_processor_gpu_batch_equals_reference(procs):
    import chain_harness as H
    cpu, gpu = procs
    rng = np.random.default_rng(77)
    pdus, weights, tbs, rb = [], [], [], 0
    for i in range(10):
        L = int(rng.integers(1, 5))
        nrb = int(rng.choice([6, 9, 16, 25]))
        qm, rate = [(8, 948.0), (6, 772.0)][i % 2]
        p = H.params(rnti=0x5000 + i, nof_rb=nrb, rb_start=rb, qm=qm, target_code_rate=rate, nof_layers=L,
                     nof_ports=P, start_symbol=2, nof_symbols=12, dmrs_mask=(1 << 2) | (1 << 11))
        rb += nrb
        seg = grant(p).segmentation()
        p.base_graph = seg.base_graph
        pdus.append(p)
        w = (rng.normal(size=(P, L)) + 1j * rng.normal(size=(P, L))) / np.sqrt(2 * L)
        weights.append(w.astype(np.complex64))
        tbs.append(rng.integers(0, 256, seg.tbs // 8).astype(np.uint8))
    other = bf16((rng.normal(size=(P, 14, 12 * 273)) + 1j * rng.normal(size=(P, 14, 12 * 273))) * 0.1)
    for slot in (3, 4):
        ref = cpu.dl_slot(slot, pdus, weights, tbs, other)
        before = gpu.pdsch_transfer_counters()
        got = gpu.dl_slot(slot, pdus, weights, tbs, other)
        after = gpu.pdsch_transfer_counters()
        assert np.array_equal(ref, got), (slot, int(np.sum(np.any(ref != got, axis=-1))))
        # One device-to-host grid transfer per slot whatever the number of devices; with three PDSCH shards (RNTI mod 3)
        # the two non-root ones merge only their UEs' subcarrier bands into the root's grid.
        assert after["grid_downloads"] - before["grid_downloads"] == 1, (before, after)
        if gpu.mode.startswith("multi3"):
            assert after["shard_merges"] - before["shard_merges"] == 2, (before, after)
            moved = after["merge_bytes"] - before["merge_bytes"]
            assert 0 < moved < 2 * P * 14 * 12 * 273 * 4, moved
        assert np.mean(np.any(ref != other, axis=-1)) > 0.3  # the PDSCHs were written
        assert np.array_equal(ref[:, :2], other[:, :2])  # symbols 0-1 (another channel's) untouched


def test_uplink_processor_gpu_batch_interpolate_equals_reference():
    """The estimator's "interpolate" time strategy (the batch keeps per-symbol estimates, DC zeroing per symbol) against
    the reference's processors with the same strategy: 10 UEs plus one over the DC subcarrier."""
    import chain_harness as H
    cpu = H.UpperPhy(0, H.UL_CPU + 2, P)
    gpu = H.UpperPhy(0, H.UL_GPU_BATCH + 2, P)
    chain = H.Chain(0)
    try:
        rng = np.random.default_rng(31)
        ues, rb = ul_ues(rng, H, 0x4a01, 10, 0)
        dc = H.params(rnti=0x4b00, harq_id=20, nof_rb=10, rb_start=rb, qm=6, target_code_rate=772.0, nof_ports=P,
                      dc_position=12 * (rb + 3) + 5)
        ues.append((dc, -40.0, 0.5, 0.0))
        tbs, sizes = [], []
        for p, *_ in ues:
            seg = grant(p).segmentation()
            p.base_graph = seg.base_graph
            tbs.append(rng.integers(0, 256, seg.tbs // 8).astype(np.uint8))
            sizes.append(seg.tbs // 8)
        grid = received_grid(rng, chain, ues, tbs, 28.0)
        pdus = [p for p, *_ in ues]
        ref = cpu.ul_slot(7, pdus, sizes, grid)
        got = gpu.ul_slot(7, pdus, sizes, grid)
        check_equal(ref, got, "interpolate")
        assert sum(d["tb_crc_ok"] for d, _ in ref) >= len(pdus) - 1
    finally:
        chain.close()
        cpu.close()
        gpu.close()


def test_gpu_factories_pdu_validators_equal_reference():
    """Row b8: create_pdu_validator() of the GPU uplink / downlink processor factories answers like the reference's
    pusch_processor_validator_impl (channel-estimate dimensions 273 PRB x 14 symbols x 4 layers x 4 ports) and
    pdsch_processor_validator_impl, message for message, on valid PDUs and on PDUs each validator rejects."""
    import chain_harness as H
    ul = [H.params(), H.params(nof_rb=273), H.params(nof_layers=2, nof_ports=4),
          H.params(nof_ports=5),                       # more rx ports than the channel-estimate dimensions
          H.params(nof_layers=5),                      # more layers
          H.params(rb_start=270, nof_rb=10),           # allocation outside the BWP
          H.params(start_symbol=10, nof_symbols=8),    # symbols past the slot
          H.params(dmrs_mask=0)]                       # no DM-RS symbol
    res = H.factory_validate(0, 0, ul)
    assert [r[:2] for r in res] == [(r[1], r[1]) for r in res], res  # same verdict as the reference
    assert not any(r[2] for r in res), res                          # same messages
    assert [r[1] for r in res][:3] == [True] * 3 and not all(r[1] for r in res), res
    dl = [H.params(nof_layers=1), H.params(nof_layers=4, nof_rb=100), H.params(nof_layers=2, start_symbol=13,
                                                                               nof_symbols=4)]
    w = [np.ones((P, p.nof_layers), np.complex64) for p in dl]
    res = H.factory_validate(0, 1, dl, w)
    assert [r[:2] for r in res] == [(r[1], r[1]) for r in res], res
    assert not any(r[2] for r in res), res


def test_dl_grid_twin_equals_downloaded_grid():
    """du_low DL with the grid's PDSCH part kept on the GPU (integration/gpu_staging.h dl_grid_twins; verdict item 5's
    DL half): one sector's GPU downlink processor (PDSCH slot batch) hands each slot's grid to the GPU PDxCH processor
    through the reference's gateway path (downlink_processor_single_executor_impl.cpp:268 send_resource_grid ->
    pdxch handle_request). With the twin the batch leaves its PDSCH REs in HBM (no download, no host store) and the
    PDxCH modulates them merged with the REs the host wrote into the grid (symbols 0-1 and the PRBs above the PDSCH,
    random); without it the batch downloads the REs into the host grid as the reference's PDSCH processor writes them.
    The baseband samples of every slot, symbol and port are equal, and the counters show which path ran (the first slot
    precedes the PDxCH's subscription, so it downloads)."""
    import ctypes

    import chain_harness as H

    lib = ctypes.CDLL(H.CHAIN_SO)
    f = lib.chain_dl_twin_samples
    f.restype = ctypes.c_int
    f.argtypes = ([ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_int, ctypes.POINTER(H.ChainParams)] +
                  [ctypes.c_void_p] * 3 + [ctypes.c_uint] * 3 + [ctypes.c_void_p] * 2)
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rng = np.random.default_rng(11)
    tbs = sch.tbs_calculate(270, 12, 6 * 3 * 2, 0, 8, 948.0, 4)
    pdu = H.params(slot=0, rnti=1, n_id=0, scrambling_id=0, nof_rb=270, rb_start=0, bwp_size=273, qm=8,
                   target_code_rate=948.0, nof_layers=4, nof_ports=4, start_symbol=2, nof_symbols=12,
                   dmrs_mask=(1 << 2) | (1 << 7) | (1 << 11), base_graph=sch.base_graph(tbs, 948 / 1024),
                   tbs_lbrm_bytes=159749)
    q, _ = np.linalg.qr(rng.normal(size=(4, 4)) + 1j * rng.normal(size=(4, 4)))
    w = np.ascontiguousarray(q.astype(np.complex64).ravel()).view(np.float32)
    tbb = np.array([tbs // 8], np.int32)
    data = rng.integers(0, 256, int(tbb.sum())).astype(np.uint8)
    arr = (H.ChainParams * 1)(pdu)
    slots = 4
    res = {}
    for twin in (0, 1):
        out = np.zeros(slots * P * 61440 * 2, np.float32)
        cnt = np.zeros(3, np.uint64)
        r = f(0, twin, slots, 1, arr, ptr(w), ptr(data), ptr(tbb), P, 273, 4096, ptr(out), ptr(cnt))
        assert r == 0, r
        res[twin] = (out, cnt)
    (ref, c0), (got, c1) = res[0], res[1]
    assert int(c0[0]) == slots and int(c0[1]) == 0, c0   # every slot downloaded
    assert int(c1[1]) == slots - 1 and int(c1[0]) == 1, c1  # all but the first through the twin
    assert int(c0[2]) == 0 and int(c1[2]) == 0
    assert np.abs(ref).max() > 0
    np.testing.assert_array_equal(got, ref)
