"""Signal-chain drop-in on the GPU: the reference's OWN processors (pusch_processor_impl, pdsch_processor_impl, compiled
from its sources by oracle/build_chain.sh) run once on the reference's CPU components and once with the GPU bindings a
maintainer adds (integration/pusch_chain_gpu.cpp, pdsch_chain_gpu.cpp, ofdm_gpu.cpp, plus the HAL accelerators)
plugged in through the same interfaces, on the same inputs (tests/chain_harness.py):

  * PUSCH processor (estimate -> demultiplex -> demodulate -> decode, pusch_processor_impl.cpp:217-:335): GPU DM-RS
    estimator + GPU demodulator with the reference CPU decoder, and with pusch_decoder_hw_impl over the GPU
    accelerator, against the all-CPU processor. Equal: TB CRC flag, TB bytes, number of codeblocks, HARQ-ACK status
    and payload. Within stated tolerances (the GPU LLRs equal the reference's or differ by one quantisation step,
    tests/test_pusch_demodulator_gpu.py): LDPC mean iterations +-0.5, post-equalisation SINR 0.1 dB, EVM 2e-3, TA 2 Tc,
    CFO 0.05 Hz, EPRE / RSRP 0.01 dB. Received grids: the reference's own transmitter (PDSCH encoder / modulator /
    DM-RS: the PUSCH scrambling, modulation and DM-RS are the PDSCH ones) through a random flat channel per rx port with
    a delay, a CFO and AWGN.
  * PDSCH processor (encode -> modulate -> DM-RS, pdsch_processor_impl.cpp:123-:153): the HW encoder over the GPU
    accelerator + GPU modulator + GPU DM-RS against the CPU processor: resource grids bit-exact, including every RE
    outside the PDSCH (pre-filled with other content) left as it was.
  * OFDM slot modulator / demodulator bindings against the reference's (generic DFT): samples within 2e-5 x RMS, grid
    values within one bf16 ulp.
"""
import numpy as np
import pytest

from ofdm_oracle import bf16_to_complex
from pusch_demod_cases import bf16
from srsgpu import sch

pytestmark = pytest.mark.gpu

T_C = 1.0 / (480000 * 4096)


@pytest.fixture(scope="module")
def chain():
    import chain_harness
    c = chain_harness.Chain(0)
    yield c
    c.close()


def ue_grant(p):
    nd = bin(p.dmrs_mask).count("1")
    return sch.UeGrant(p.nof_rb, p.nof_layers, p.qm, p.target_code_rate, nof_symb_sh=p.nof_symbols,
                       nof_dmrs_symbols=nd)


def receive(rng, tx, nof_ports, snr_db, cfo_hz=0.0, delay=0.0):
    """tx (L, 14, nsc, 2) bf16 -> rx (P, 14, nsc, 2): a random complex gain per (port, layer) with a common delay
    (phase ramp, in samples of a 4096-point DFT), a CFO (symbol l rotated by 2 pi cfo t_l) and AWGN."""
    import pusch_chest_oracle as C
    x = bf16_to_complex(tx)
    L, _, nsc = x.shape
    k = np.arange(nsc)
    g = (rng.normal(size=(nof_ports, L)) + 1j * rng.normal(size=(nof_ports, L))) / np.sqrt(2 * L)
    ramp = np.exp(-2j * np.pi * k * delay / 4096)
    y = np.einsum("pl,lsk->psk", g, x) * ramp[None, None, :]
    if cfo_hz:
        ep = C.symbol_start_epochs(1)
        y = y * np.exp(2j * np.pi * cfo_hz / 30000.0 * ep)[None, :, None]
    nv = 10 ** (-snr_db / 10)
    y = y + (rng.normal(size=y.shape) + 1j * rng.normal(size=y.shape)) * np.sqrt(nv / 2)
    return bf16(y)


def check_pusch_equal(ref, got, what):
    tb_r, r = ref
    tb_g, g = got
    assert g["sch"] == 1 and r["sch"] == 1, what
    assert g["tb_crc_ok"] == r["tb_crc_ok"], (what, r, g)
    assert g["nof_cbs"] == r["nof_cbs"], what
    if r["tb_crc_ok"]:
        assert np.array_equal(tb_g, tb_r), what
    if r["ldpc_obs"] > 0:
        assert abs(g["ldpc_mean"] - r["ldpc_mean"]) <= 0.5, (what, r["ldpc_mean"], g["ldpc_mean"])
    assert abs(g["sinr_db"] - r["sinr_db"]) < 0.1, (what, r["sinr_db"], g["sinr_db"])
    assert abs(g["evm"] - r["evm"]) < 2e-3, (what, r["evm"], g["evm"])
    assert abs(g["ta_s"] - r["ta_s"]) <= 2 * T_C, (what, r["ta_s"], g["ta_s"])
    if not np.isnan(r["cfo_hz"]):
        assert abs(g["cfo_hz"] - r["cfo_hz"]) < 0.05, (what, r["cfo_hz"], g["cfo_hz"])
    assert abs(g["epre_db"] - r["epre_db"]) < 0.01 and abs(g["rsrp_db"] - r["rsrp_db"]) < 0.01, (what, r, g)
    assert g["uci"] == r["uci"], what
    if r["uci"]:
        assert g["harq_ack_status"] == r["harq_ack_status"] and g["harq_ack_bits"] == r["harq_ack_bits"], (what, r, g)


PUSCH_CASES = [
    # (description, params overrides, snr dB, cfo Hz, delay samples)
    ("25 PRB 256QAM MCS27 pos1", dict(nof_rb=25, rb_start=10, qm=8, target_code_rate=948.0), 32.0, 150.0, 3.0),
    ("51 PRB 64QAM pos1 slot 3", dict(nof_rb=51, rb_start=100, qm=6, target_code_rate=772.0, slot=3), 24.0, -80.0,
     -2.0),
    ("4 PRB 256QAM one DM-RS", dict(nof_rb=4, rb_start=0, dmrs_mask=1 << 2), 30.0, 0.0, 1.0),
    ("273 PRB 256QAM (configs[4] UL)", dict(nof_rb=273, rb_start=0, qm=8, target_code_rate=948.0), 30.0, 200.0, 4.0),
    ("100 PRB 16QAM 2 rx ports, DC", dict(nof_rb=100, rb_start=50, qm=4, target_code_rate=616.0, nof_ports=2,
                                          dc_position=12 * 136 + 6), 18.0, 40.0, 0.0),
    ("20 PRB 64QAM low SNR (fails)", dict(nof_rb=20, rb_start=30, qm=6, target_code_rate=873.0), 9.0, 0.0, 0.0),
    ("12 PRB QPSK 11 symbols, HARQ-ACK 2 bits", dict(nof_rb=12, rb_start=5, qm=2, target_code_rate=308.0,
                                                      start_symbol=2, nof_symbols=11, dmrs_mask=(1 << 3) | (1 << 9),
                                                      nof_harq_ack=2), 15.0, 60.0, 0.0),
]


@pytest.mark.parametrize("mode", [1, 2])
def test_pusch_processor_gpu_chain_equals_reference(chain, mode):
    import chain_harness as H
    rng = np.random.default_rng(40 + mode)
    for i, (what, over, snr, cfo, delay) in enumerate(PUSCH_CASES):
        p = H.params(harq_id=i, **over)
        seg = ue_grant(p).segmentation()
        p.base_graph = seg.base_graph
        tb = rng.integers(0, 256, seg.tbs // 8).astype(np.uint8)
        rx = receive(rng, chain.ue_tx(p, tb), p.nof_ports, snr, cfo, delay)
        ref = chain.pusch(H.PUSCH_CPU, p, rx, seg.tbs // 8)
        got = chain.pusch(mode, p, rx, seg.tbs // 8)
        check_pusch_equal(ref, got, what)
        if "fails" not in what and p.nof_harq_ack == 0:
            assert ref[1]["tb_crc_ok"] == 1 and np.array_equal(ref[0], tb), what


def test_pusch_processor_gpu_chain_harq_retransmission(chain):
    """rv0 too noisy to decode alone, then rv2 (new_data = false) combines with it: the GPU chain with the HW decoder
    (HARQ in HBM) and with the CPU decoder give the reference's outcomes. (A process whose rv0 decodes is released by
    the reference, pusch_decoder_hw_impl.cpp:411: its retransmission is not a combining case and is skipped.)"""
    import chain_harness as H
    rng = np.random.default_rng(47)
    outcomes = []
    for h, snr in enumerate((5.0, 5.5, 6.0, 6.5, 7.0, 7.5)):
        kw = dict(nof_rb=30, rb_start=40, qm=6, target_code_rate=772.0, harq_id=100 + h)
        seg = ue_grant(H.params(**kw)).segmentation()
        tb = rng.integers(0, 256, seg.tbs // 8).astype(np.uint8)
        for rv, new_data in ((0, 1), (2, 0)):
            p = H.params(rv=rv, new_data=new_data, base_graph=seg.base_graph, **kw)
            rx = receive(rng, chain.ue_tx(p, tb), 4, snr)
            ref = chain.pusch(H.PUSCH_CPU, p, rx, seg.tbs // 8)
            for mode in (1, 2):
                check_pusch_equal(ref, chain.pusch(mode, p, rx, seg.tbs // 8), (h, rv, mode))
            outcomes.append((h, rv, ref[1]["tb_crc_ok"]))
            if ref[1]["tb_crc_ok"]:
                break
    assert any(ok for (_, rv, ok) in outcomes if rv == 2), outcomes


PDSCH_CASES = [
    ("configs[1]: 51 PRB SISO 64QAM", dict(nof_rb=51, rb_start=0, bwp_size=51, grid_prb=51, qm=6,
                                           target_code_rate=772.0, nof_layers=1, nof_ports=1, dmrs_mask=1 << 2)),
    ("100 MHz 4 layers 256QAM pos1", dict(nof_rb=273, rb_start=0, qm=8, target_code_rate=948.0, nof_layers=4,
                                          nof_ports=4)),
    # Type 1 only at the processor level: pdsch_processor_impl::modulate never sets the modulator's dmrs_config_type
    # (pdsch_processor_impl.cpp:180-196), so a type-2 PDU reaches the modulator as type 1 (reference defect; the GPU
    # modulator's type-2 mapping is pinned at component level, tests/test_pdsch_modulator_gpu.py).
    ("2 layers on 4 ports, offset, 1 CDM group (data on DM-RS symbols)",
     dict(nof_rb=40, rb_start=17, qm=4, target_code_rate=616.0, nof_layers=2, nof_ports=4, cdm_groups=1,
          start_symbol=1, nof_symbols=12, dmrs_mask=(1 << 2) | (1 << 8))),
    ("special slot: 8 symbols DM-RS 2+7", dict(nof_rb=273, rb_start=0, qm=8, target_code_rate=948.0, nof_layers=4,
                                               nof_ports=4, nof_symbols=8, dmrs_mask=(1 << 2) | (1 << 7))),
]


def test_pdsch_processor_gpu_chain_equals_reference(chain):
    import chain_harness as H
    rng = np.random.default_rng(50)
    for what, over in PDSCH_CASES:
        p = H.params(**over)
        nd = bin(p.dmrs_mask).count("1")
        # Data REs per PRB on DM-RS symbols: 12 - 6 x CDM groups (type 1) / 4 x (type 2).
        dre = 12 - p.cdm_groups * (4 if p.dmrs_type2 else 6)
        tbs = sch.tbs_calculate(p.nof_rb, p.nof_symbols, (12 - dre) * nd, 0, p.qm, p.target_code_rate, p.nof_layers)
        p.base_graph = sch.base_graph(tbs, p.target_code_rate / 1024)
        tb = rng.integers(0, 256, tbs // 8).astype(np.uint8)
        w = (rng.normal(size=(p.nof_ports, p.nof_layers)) + 1j * rng.normal(size=(p.nof_ports, p.nof_layers))) / 2
        # Other channels' content everywhere: the PDSCH processors must leave every RE they do not own untouched.
        grid0 = rng.integers(0, 1 << 16, (p.nof_ports, 14, 12 * p.grid_prb, 2)).astype(np.uint16)
        ref = chain.pdsch(H.PDSCH_CPU, p, w, tb, grid0)
        got = chain.pdsch(H.PDSCH_GPU, p, w, tb, grid0)
        diff = np.flatnonzero(np.any(ref != got, axis=-1))
        assert diff.size == 0, (what, diff[:10], diff.size)
        assert np.mean(np.any(ref != grid0, axis=-1)) > 0.05, what  # the PDSCH was written


@pytest.mark.parametrize("slot", [0, 1])
def test_ofdm_bindings_equal_reference(chain, slot):
    rng = np.random.default_rng(60 + slot)
    bw, N = 273, 4096
    x = (rng.normal(size=(1, 14, 12 * bw)) + 1j * rng.normal(size=(1, 14, 12 * bw))) * 0.3
    grid = bf16(x)
    a = chain.ofdm_modulate(0, grid, 1, bw, N, 1.0 / 64, 3.5e9, slot)
    b = chain.ofdm_modulate(1, grid, 1, bw, N, 1.0 / 64, 3.5e9, slot)
    assert a.shape == b.shape
    rms = np.sqrt(np.mean(np.abs(a) ** 2))
    assert np.max(np.abs(a - b)) < 2e-5 * rms, np.max(np.abs(a - b)) / rms
    ga = chain.ofdm_demodulate(0, a, 1, bw, N, 1.0 / (N / 64), 3.5e9, slot, window_offset=72)
    gb = chain.ofdm_demodulate(1, a, 1, bw, N, 1.0 / (N / 64), 3.5e9, slot, window_offset=72)
    # Within one bf16 ulp (2^-7 relative) or 1e-4 x RMS absolute (tests/test_ofdm_gpu.py's tolerance).
    va, vb = bf16_to_complex(ga), bf16_to_complex(gb)
    ref_rms = np.sqrt(np.mean(np.abs(va) ** 2))
    err = np.abs(va - vb)
    assert np.all(err <= np.maximum(2.0 ** -7 * np.abs(va), 1e-4 * ref_rms)), float(np.max(err / ref_rms))
