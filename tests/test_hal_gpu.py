"""Processor / HAL-level drop-in on the GPU: the reference's OWN transport-block processors (compiled from its sources
by oracle/build_hal.sh) drive the MI355X through the bindings a maintainer adds (integration/), and their results are
compared with the reference's CPU processors on the same inputs, through the same harness (tests/hal_lib.py):

  * pusch_decoder_hw_impl over hal::hw_accelerator_pusch_dec (integration/hw_accelerator_pusch_dec_gpu.cpp, HARQ soft
    buffers in HBM) and pusch_decoder_impl with the GPU ldpc_decoder (integration/ldpc_decoder_gpu.cpp) against
    pusch_decoder_impl with the reference's AVX-512 / AVX2 decoder: TB bytes, TB CRC flag and the LDPC iteration
    statistics (count, min, max, mean) equal, new transmissions and rv2 retransmissions (HARQ combining);
  * pdsch_encoder_hw_impl over hal::hw_accelerator_pdsch_enc (integration/hw_accelerator_pdsch_enc_gpu.cpp) against
    pdsch_encoder_impl (AVX2 encoder): codewords bit-exact.

Grants: random TB sizes (CRC16 / CRC24A single-codeblock, CRC24B segmented, BG1 / BG2), BASELINE configs[1] (20 MHz
SISO 64QAM PDSCH) and configs[2] (100 MHz 2x2 256QAM PUSCH) and the bench slot's UE grants."""
import numpy as np
import pytest

from chain_lib import bits_to_llrs, oracle_pdsch_encode
from oracle_lib import Oracle
from srsgpu import sch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hal():
    import hal_lib
    h = hal_lib.Hal(0)
    yield h
    h.close()


def grants(rng):
    tables = list(sch.MCS_TABLE_256QAM.values())
    out = []
    for _ in range(24):
        qm, r = tables[int(rng.integers(0, len(tables)))]
        out.append(sch.UeGrant(int(rng.integers(1, 60)), int(rng.integers(1, 5)), qm, r,
                               nof_symb_sh=int(rng.integers(4, 15))))
    out += sch.slot_100mhz_4x4(nof_ues=8, nof_prb=51, nof_layers=1, mcs=20)       # configs[1]-like: SISO, 64QAM
    out += sch.slot_100mhz_4x4(nof_ues=4, nof_prb=273, nof_layers=2, mcs=27)[:4]  # configs[2]: 100 MHz 2x2 256QAM
    out += sch.slot_100mhz_4x4(nof_layers=1, nof_dmrs_symbols=2)[:6]             # the bench slot's UL grants
    return out


def test_hal_pusch_decoder_gpu_equals_reference_cpu(hal):
    import hal_lib
    orc = Oracle()
    rng = np.random.default_rng(21)
    gs = grants(rng)
    n_ok = 0
    for i, g in enumerate(gs):
        seg = g.segmentation()
        tb = rng.integers(0, 256, seg.tbs // 8).astype(np.uint8)
        noise = [0.0, 5.0, 8.0, 11.0][i % 4]
        for rv, new_data in ((0, True), (2, False)):
            cw, _, _ = oracle_pdsch_encode(orc, tb, seg.base_graph, rv, g.qm, g.nof_layers, 0, g.nof_ch_symbols)
            llr = bits_to_llrs(rng, cw, amp=6.0, noise=noise)
            res = [hal.pusch_decode(m, i, seg.nof_segments, seg.base_graph, rv, g.qm, g.nof_layers, llr, seg.tbs // 8,
                                    new_data=new_data)
                   for m in (hal_lib.PUSCH_CPU, hal_lib.PUSCH_SW_GPU_LDPC, hal_lib.PUSCH_HW_GPU)]
            (tb0, s0), (tb1, s1), (tb2, s2) = res
            assert s1 == s0, (i, rv, s0, s1)
            assert s2 == s0, (i, rv, s0, s2)
            if s0["tb_crc_ok"]:
                assert np.array_equal(tb0, tb) and np.array_equal(tb1, tb) and np.array_equal(tb2, tb), (i, rv)
                n_ok += 1
    assert n_ok >= 20


def test_hal_pdsch_encoder_gpu_equals_reference_cpu(hal):
    import hal_lib
    rng = np.random.default_rng(22)
    for i, g in enumerate(grants(rng)):
        seg = g.segmentation()
        tb = rng.integers(0, 256, seg.tbs // 8).astype(np.uint8)
        rv = i % 4
        Nref = 0 if i % 3 else (seg.segment_length + (66 if seg.base_graph == 1 else 50) * seg.lifting_size) // 2
        a = hal.pdsch_encode(hal_lib.PDSCH_CPU, seg.base_graph, rv, g.qm, g.nof_layers, g.nof_ch_symbols, tb, Nref)
        b = hal.pdsch_encode(hal_lib.PDSCH_HW_GPU, seg.base_graph, rv, g.qm, g.nof_layers, g.nof_ch_symbols, tb, Nref)
        assert np.array_equal(a, b), (i, seg.tbs, seg.nof_segments, rv, Nref)


def test_hal_pusch_decoder_thread_pool_shares_harq():
    """The reference's thread-pool wiring of the HW decoder (pusch_decoder_factory_hw, factories.cpp:122-140): a
    temporary accelerator factory (destroyed before decoding) makes 4 accelerators in one hw_decoder_pool; 4 worker
    threads each own a pusch_decoder_hw_impl. Every HARQ process sends rv0 (too noisy to decode alone for most) on one
    thread and its rv2 retransmission on ANOTHER thread, i.e. another accelerator; processes interleave. The combined
    results (TB bytes, CRC, LDPC iteration statistics) equal the reference CPU decoder's on the same sequence."""
    import hal_lib
    orc = Oracle()
    rng = np.random.default_rng(31)
    pool = hal_lib.HalPool(0, max_cb_ids=64 * 160, nof_threads=4)
    try:
        gs = sch.slot_100mhz_4x4(nof_layers=1, nof_dmrs_symbols=2)[:6] + \
            sch.slot_100mhz_4x4(nof_ues=2, nof_prb=273, nof_layers=2, mcs=27)[:2]
        jobs = []
        for h, g in enumerate(gs):
            seg = g.segmentation()
            tb = rng.integers(0, 256, seg.tbs // 8).astype(np.uint8)
            llrs = []
            for rv in (0, 2):
                cw, _, _ = oracle_pdsch_encode(orc, tb, seg.base_graph, rv, g.qm, g.nof_layers, 0, g.nof_ch_symbols)
                llrs.append(bits_to_llrs(rng, cw, amp=6.0, noise=[3.5, 4.5, 5.5][h % 3]))
            jobs.append((h, g, seg, tb, llrs))
        # All first transmissions, then all retransmissions, each on a thread other than the first one's.
        ok = {}
        for step, (rv, new_data) in enumerate(((0, True), (2, False))):
            for h, g, seg, tb, llrs in jobs:
                if step == 1 and ok[(h, 0)]:
                    continue  # decoded and released at rv0: not a combining case (pusch_decoder_hw_impl.cpp:411)
                worker = (h + 2 * step) % 4
                args = (h, seg.nof_segments, seg.base_graph, rv, g.qm, g.nof_layers, llrs[step], seg.tbs // 8)
                tb_gpu, s_gpu = pool.decode(worker, *args, new_data=new_data)
                tb_cpu, s_cpu = pool.decode(-1, *args, new_data=new_data)
                assert s_gpu == s_cpu, (h, rv, s_cpu, s_gpu)
                if s_cpu["tb_crc_ok"]:
                    assert np.array_equal(tb_gpu, tb) and np.array_equal(tb_cpu, tb), (h, rv)
                ok[(h, step)] = s_cpu["tb_crc_ok"]
        # Combining happened: some processes fail alone at rv0 and decode after the rv2 retransmission.
        assert sum(not ok[(h, 0)] and ok.get((h, 1), False) for h in range(len(jobs))) >= 1, ok
        # free_harq_context_entry (called by the reference once the TB CRC passes): a later retransmission into the
        # released entries combines like a new soft buffer, i.e. exactly as into identifiers never used before
        # (ext_harq_buffer_context_repository::get resets a freed entry).
        h, g, seg, tb, llrs = next(j for j in jobs if ok.get((j[0], 1), False))
        args = (seg.nof_segments, seg.base_graph, 2, g.qm, g.nof_layers, llrs[1], seg.tbs // 8)
        tb_a, s_a = pool.decode(1, h, *args, new_data=False)
        tb_b, s_b = pool.decode(3, 60, *args, new_data=False)
        assert s_a == s_b and np.array_equal(tb_a, tb_b), (s_a, s_b)
    finally:
        pool.close()


def test_hal_accelerator_rejected_codeblock_keeps_the_others_results():
    """A codeblock the accelerator rejects at enqueue (here an oversized rate-matched span) is reported as failed, and
    every other codeblock of the TB still reports ITS OWN CRC flag, iteration count and message: the plan numbers only
    the accepted codeblocks, so the results are scattered back to their operations
    (integration/hw_accelerator_pusch_dec_gpu.cpp run(); round-4 ADVICE). The first of four codeblocks is rejected;
    the last one is noisy enough to need more iterations than the clean ones, so a shifted read would show."""
    import ctypes
    import hal_lib
    orc = Oracle()
    rng = np.random.default_rng(5)
    g = sch.UeGrant(100, 1, 6, 772.0, nof_dmrs_symbols=2)
    seg = g.segmentation()
    assert seg.base_graph == 1 and seg.nof_segments >= 3
    tb = rng.integers(0, 256, seg.tbs // 8).astype(np.uint8)
    cw, _, _ = oracle_pdsch_encode(orc, tb, 1, 0, g.qm, 1, 0, g.nof_ch_symbols)
    n = seg.nof_segments
    parts = []
    for cb in seg.codeblocks:
        bits = cw[cb.cw_offset:cb.cw_offset + cb.rm_length]
        noise = 3.5 if cb.index == n - 1 else 0.0
        parts.append(bits_to_llrs(rng, bits, amp=8.0, noise=noise))
    llrs = np.concatenate(parts)
    lib = ctypes.CDLL(hal_lib.HAL_SO)
    P = ctypes.c_void_p
    lib.hal_accel_decode_ops.restype = ctypes.c_int
    lib.hal_accel_decode_ops.argtypes = [ctypes.c_int] + [ctypes.c_uint] * 4 + [P] * 6 + [ctypes.c_uint]
    E = np.array([cb.rm_length for cb in seg.codeblocks], np.uint32)

    def run(reject):
        rej = np.array(reject, np.uint8)
        crc = np.zeros(n, np.int32)
        its = np.zeros(n, np.int32)
        msgs = np.zeros((n, 1056), np.uint8)
        ptr = lambda a: a.ctypes.data_as(P)  # noqa: E731
        assert lib.hal_accel_decode_ops(0, n, seg.lifting_size, seg.nof_filler_bits, g.qm, ptr(E), ptr(llrs), ptr(rej),
                                        ptr(crc), ptr(its), ptr(msgs), 1056) == 0
        return crc, its, msgs

    crc0, its0, msgs0 = run([0] * n)
    assert crc0.all() and its0[-1] > its0[0], (crc0, its0)
    crc1, its1, msgs1 = run([1] + [0] * (n - 1))
    assert crc1[0] == 0 and its1[0] == 6, (crc1, its1)
    assert np.array_equal(crc1[1:], crc0[1:]) and np.array_equal(its1[1:], its0[1:]), (crc0, its0, crc1, its1)
    assert np.array_equal(msgs1[1:], msgs0[1:])
