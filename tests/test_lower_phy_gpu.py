"""Lower-PHY drop-in (row b5): the objects du_low's radio unit drives per OFDM symbol (lib/ru/generic/lower_phy/
lower_phy_factory.cpp:70/:84) on the GPU.

The same scripted sequence of upper-PHY requests (handle_request with a resource grid for a slot) and baseband symbols
(process_symbol) drives (tests/lower_harness.py, oracle/ref/ref_lower.cpp):
  * the reference's own pdxch_processor_impl / puxch_processor_impl, compiled from its sources, on the reference's OFDM
    symbol (de)modulator with the generic DFT (the CPU path);
  * the same reference processors on the GPU symbol objects of integration/ofdm_gpu.cpp (the factories'
    create_ofdm_symbol_(de)modulator no longer return nullptr);
  * the GPU PDxCH / PUxCH processors of integration/lower_phy_gpu.cpp (whole-slot modulation at request time;
    asynchronous per-symbol demodulation with 0 or more symbols in flight).
Equal across all: process_symbol's return value per symbol, the late-request notifications and (UL) the sequence of
received-symbol notifications. Samples within 2e-5 x RMS of the reference (tests/test_ofdm_gpu.py's bound), the buffer
left untouched exactly where the reference leaves it; grid values within one bf16 ulp (or 1e-4 x RMS), and untouched
REs untouched. The scripts cover requests for every slot, missing requests, empty grids, empty ports, a request
overwritten by one 16 slots later (late), a request processed 16 slots late, partial slots and a slot left mid-way.
"""
import numpy as np
import pytest

from lower_harness import (GPU_GROUP, GPU_GROUP_MAPPED, GPU_PROCESSOR, PROCESS, REF_CPU, REF_ON_GPU_SYMBOLS, REQUEST, SENTINEL, Lower,
                           symbol_size)
from ofdm_oracle import bf16_to_complex
from pusch_demod_cases import bf16

pytestmark = pytest.mark.gpu

CONFIGS = {
    "100MHz_30kHz_4port": dict(numerology=1, bw_rb=273, dft_size=4096, extended=False, center_freq_hz=3.5e9,
                               nof_ports=4, window_offset=0.5),
    "10MHz_15kHz_2port": dict(numerology=0, bw_rb=52, dft_size=1024, extended=False, center_freq_hz=1.8e9,
                              nof_ports=2, window_offset=0.0),
    "60kHz_extended_cp": dict(numerology=2, bw_rb=24, dft_size=512, extended=True, center_freq_hz=3.0e9,
                              nof_ports=1, window_offset=0.25),
}


@pytest.fixture(scope="module")
def lower():
    return Lower()


def dl_script(nsymb):
    """Requests and symbols: (kind, system slot, a, b)."""
    B = 40  # first system slot (any)
    ev = [(REQUEST, B + 3, 0, 0), (REQUEST, B + 4, 1, 0), (REQUEST, B + 5, 2, 0), (REQUEST, B + 6, 3, 0),
          (REQUEST, B + 6 + 16, 4, 0),   # overwrites slot B+6's entry: late B+6
          (REQUEST, B + 9, 5, 0)]
    ev += [(PROCESS, B + s, 0, nsymb) for s in (2, 3, 4, 5, 6)]  # B+2: no request; B+5: empty grid; B+6: late B+22
    ev += [(REQUEST, B + 7, 6, 0), (PROCESS, B + 7, 0, 5),      # a partial slot
           (REQUEST, B + 8, 7, 0), (PROCESS, B + 8, 3, nsymb),  # a slot entered mid-way
           (PROCESS, B + 9 + 16, 0, 2)]                         # slot B+9's request found 16 slots late
    return ev


def dl_grids(rng, cfg, nsymb, n=8):
    P, nsc = cfg["nof_ports"], 12 * cfg["bw_rb"]
    x = (rng.normal(size=(n, P, nsymb, nsc)) + 1j * rng.normal(size=(n, P, nsymb, nsc))) * 0.25
    mask = np.full(n, (1 << P) - 1, np.uint32)
    mask[1] = 0b0101 & ((1 << P) - 1) if P > 1 else 1  # empty ports
    mask[2] = 0                                        # an empty grid: nothing to transmit
    return bf16(x), mask


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_pdxch_processor_gpu_equals_reference(lower, name):
    cfg = CONFIGS[name]
    nsymb = 12 if cfg["extended"] else 14
    grids, mask = dl_grids(np.random.default_rng(7), cfg, nsymb)
    ev = dl_script(nsymb)
    ref, ref_flags, ref_late = lower.pdxch(REF_CPU, cfg, grids, mask, ev)
    assert ref_flags.any() and not ref_flags.all() and ref_late, "the script exercises every branch"
    touched = ref.real != SENTINEL
    rms = np.sqrt(np.mean(np.abs(ref[touched]) ** 2))
    for variant in (REF_ON_GPU_SYMBOLS, GPU_PROCESSOR):
        got, flags, late = lower.pdxch(variant, cfg, grids, mask, ev)
        assert np.array_equal(flags, ref_flags), variant
        assert late == ref_late, variant
        assert got.shape == ref.shape
        assert np.array_equal(got.real == SENTINEL, ~touched), variant  # same buffers left untouched
        err = np.max(np.abs(got[touched] - ref[touched]))
        assert err < 2e-5 * rms, (variant, err / rms)


def ul_script(nsymb):
    B = 100
    return [(REQUEST, B + 3, 0, 0), (PROCESS, B + 2, 0, nsymb), (PROCESS, B + 3, 0, nsymb),
            (REQUEST, B + 4, 1, 0), (PROCESS, B + 4, 0, 7),          # a slot left mid-way
            (PROCESS, B + 5, 0, nsymb),                              # no request
            (REQUEST, B + 6, 2, 0), (REQUEST, B + 6 + 16, 3, 0),     # overwritten: late B+6
            (PROCESS, B + 6, 0, nsymb),                              # finds B+22: late B+22
            (REQUEST, B + 7, 4, 0), (PROCESS, B + 7, 2, nsymb),      # entered mid-way
            (REQUEST, B + 8, 5, 0), (PROCESS, B + 8, 0, nsymb)]


def ul_samples(rng, cfg, ev):
    n = sum(cfg["nof_ports"] * symbol_size(cfg["numerology"], cfg["dft_size"], cfg["extended"], e[1], l)
            for e in ev if e[0] == PROCESS for l in range(e[2], e[3]))
    return ((rng.normal(size=n) + 1j * rng.normal(size=n)) * 0.05).astype(np.complex64)


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_puxch_processor_gpu_equals_reference(lower, name):
    cfg = CONFIGS[name]
    nsymb = 12 if cfg["extended"] else 14
    ev = ul_script(nsymb)
    x = ul_samples(np.random.default_rng(11), cfg, ev)
    ref, ref_flags, ref_rx, ref_late = lower.puxch(REF_CPU, cfg, 6, ev, x)
    assert ref_flags.any() and not ref_flags.all() and ref_late and ref_rx
    va = bf16_to_complex(ref)
    rms = np.sqrt(np.mean(np.abs(va[va != 0]) ** 2))
    for variant, in_flight in ((REF_ON_GPU_SYMBOLS, 0), (GPU_PROCESSOR, 0), (GPU_PROCESSOR, 3)):
        got, flags, rx, late = lower.puxch(variant, cfg, 6, ev, x, max_in_flight=in_flight)
        what = (variant, in_flight)
        assert np.array_equal(flags, ref_flags), what
        assert rx == ref_rx, what
        assert late == ref_late, what
        vb = bf16_to_complex(got)
        assert np.array_equal(va == 0, vb == 0), what  # the same REs written
        err = np.abs(va - vb)
        assert np.all(err <= np.maximum(2.0 ** -7 * np.abs(va), 1e-4 * rms)), (what, float(np.max(err / rms)))


def test_sectors_on_one_gpu_equal_reference(lower):
    """Several sectors on one GPU, as the reference's radio unit runs them: one lower-PHY sector per cell
    (lib/ru/generic/ru_factory_generic_impl.cpp:75-90), each driven from its own thread. Every sector's PDxCH and
    PUxCH GPU processors run concurrently with the others' (own streams, graphs and staging on a shared context) and
    each equals the reference run alone on that sector's data."""
    from concurrent.futures import ThreadPoolExecutor

    sectors = [(name, seed) for seed, name in enumerate(sorted(CONFIGS) * 2)]  # 6 sectors, 3 configurations
    inputs = []
    for name, seed in sectors:
        cfg = CONFIGS[name]
        nsymb = 12 if cfg["extended"] else 14
        rng = np.random.default_rng(100 + seed)
        grids, mask = dl_grids(rng, cfg, nsymb)
        ev_ul = ul_script(nsymb)
        inputs.append((cfg, grids, mask, dl_script(nsymb), ev_ul, ul_samples(rng, cfg, ev_ul)))

    def run(variant, i):
        cfg, grids, mask, ev_dl, ev_ul, x = inputs[i]
        dl = lower.pdxch(variant, cfg, grids, mask, ev_dl)
        ul = lower.puxch(variant, cfg, 6, ev_ul, x, max_in_flight=0)
        return dl, ul

    refs = [run(REF_CPU, i) for i in range(len(sectors))]
    with ThreadPoolExecutor(len(sectors)) as pool:
        gots = list(pool.map(lambda i: run(GPU_PROCESSOR, i), range(len(sectors))))
    for (name, _), (rdl, rul), (gdl, gul) in zip(sectors, refs, gots):
        touched = rdl[0].real != SENTINEL
        rms = np.sqrt(np.mean(np.abs(rdl[0][touched]) ** 2))
        assert np.array_equal(gdl[1], rdl[1]) and gdl[2] == rdl[2], name
        assert np.array_equal(gdl[0].real == SENTINEL, ~touched), name
        assert np.max(np.abs(gdl[0][touched] - rdl[0][touched])) < 2e-5 * rms, name
        assert np.array_equal(gul[1], rul[1]) and gul[2] == rul[2] and gul[3] == rul[3], name
        va, vb = bf16_to_complex(rul[0]), bf16_to_complex(gul[0])
        rms = np.sqrt(np.mean(np.abs(va[va != 0]) ** 2))
        assert np.array_equal(va == 0, vb == 0), name
        assert np.all(np.abs(va - vb) <= np.maximum(2.0 ** -7 * np.abs(va), 1e-4 * rms)), name


@pytest.mark.parametrize("name", ["100MHz_30kHz_4port", "10MHz_15kHz_2port"])
@pytest.mark.parametrize("in_flight", [0, 3])
@pytest.mark.parametrize("variant", [GPU_GROUP, GPU_GROUP_MAPPED], ids=["staged", "mapped_ul_grids"])
def test_sector_group_equals_reference(lower, name, in_flight, variant):
    """The sector group (lower_phy_sector_group: the same symbol / slot of every sector in one launch): four sectors
    on their own carrier frequencies and data, driven from their own threads through the edge-case scripts above
    (missing requests, late and overwritten requests, partial slots, a slot left mid-way, empty grids and ports), each
    equal to the reference processor run on that sector; and the group did batch several sectors' work per launch
    (the sectors are paced at the symbol rate, as a radio unit drives them). mapped_ul_grids: the UL grids are
    mapped for the device (as the GPU uplink processor's PUSCH batch maps its grid), so the group demodulates into
    their rows directly instead of staging them (srsgpu_ofdm_jobs_execute_direct); the grids, notifications and
    empty-port marks must be the same."""
    cfg = CONFIGS[name]
    nsymb = 12 if cfg["extended"] else 14
    S, G = 4, 8
    freqs = [cfg["center_freq_hz"] + 1e7 * k for k in range(S)]
    rng = np.random.default_rng(41)
    grids, masks = zip(*(dl_grids(rng, cfg, nsymb, G) for _ in range(S)))
    grids, masks = np.stack(grids), np.stack(masks)
    ev_dl, ev_ul = dl_script(nsymb), ul_script(nsymb)
    x = np.stack([ul_samples(rng, cfg, ev_ul) for _ in range(S)])
    ref = lower.sectors(REF_CPU, cfg, freqs, grids, masks, ev_dl, ev_ul, x)
    # paced at the radio's symbol rate, as a radio unit drives its sectors: their symbols meet in the group's rounds
    got = lower.sectors(variant, cfg, freqs, grids, masks, ev_dl, ev_ul, x, max_in_flight=in_flight, paced=True)
    for k in range(S):
        (rs, rf), (gs, gf) = ref["dl"][k], got["dl"][k]
        touched = rs.real != SENTINEL
        rms = np.sqrt(np.mean(np.abs(rs[touched]) ** 2))
        assert np.array_equal(gf, rf), k
        assert np.array_equal(gs.real == SENTINEL, ~touched), k
        assert np.max(np.abs(gs[touched] - rs[touched])) < 2e-5 * rms, k
        (rg, rfl, rrx), (gg, gfl, grx) = ref["ul"][k], got["ul"][k]
        assert np.array_equal(gfl, rfl) and grx == rrx, k
        assert got["late"][k] == ref["late"][k], k
        va, vb = bf16_to_complex(rg), bf16_to_complex(gg)
        rms = np.sqrt(np.mean(np.abs(va[va != 0]) ** 2))
        assert np.array_equal(va == 0, vb == 0), k
        assert np.all(np.abs(va - vb) <= np.maximum(2.0 ** -7 * np.abs(va), 1e-4 * rms)), k
    c = got["group"]
    assert c["ul_launches"] > 0 and c["ul_batched"] > c["ul_launches"] and c["ul_batched"] > c["ul_alone"], c
    assert c["dl_launches"] > 0 and c["dl_batched"] > c["dl_launches"] and c["dl_batched"] > c["dl_alone"], c


# ref_lower.cpp group_prelude: the tested sector joins a two-sector group after another one registered first.
GROUP_FIRST_REMOVED, GROUP_FIRST_OTHER_CP = 4, 5
CONFIG_60K_NORMAL = dict(numerology=2, bw_rb=24, dft_size=512, extended=False, center_freq_hz=3.0e9, nof_ports=1,
                         window_offset=0.25)


def check_group_sector(lower, cfg, variant, seed=5):
    nsymb = 12 if cfg["extended"] else 14
    grids, mask = dl_grids(np.random.default_rng(seed), cfg, nsymb)
    ev = dl_script(nsymb)
    ref, ref_flags, ref_late = lower.pdxch(REF_CPU, cfg, grids, mask, ev)
    got, flags, late = lower.pdxch(variant, cfg, grids, mask, ev)
    touched = ref.real != SENTINEL
    rms = np.sqrt(np.mean(np.abs(ref[touched]) ** 2))
    assert np.array_equal(flags, ref_flags) and late == ref_late
    assert np.array_equal(got.real == SENTINEL, ~touched)
    assert np.max(np.abs(got[touched] - ref[touched])) < 2e-5 * rms
    ev = ul_script(nsymb)
    x = ul_samples(np.random.default_rng(seed + 1), cfg, ev)
    ref, ref_flags, ref_rx, ref_late = lower.puxch(REF_CPU, cfg, 6, ev, x)
    got, flags, rx, late = lower.puxch(variant, cfg, 6, ev, x, max_in_flight=3)
    assert np.array_equal(flags, ref_flags) and rx == ref_rx and late == ref_late
    va, vb = bf16_to_complex(ref), bf16_to_complex(got)
    rms = np.sqrt(np.mean(np.abs(va[va != 0]) ** 2))
    assert np.array_equal(va == 0, vb == 0)
    assert np.all(np.abs(va - vb) <= np.maximum(2.0 ** -7 * np.abs(va), 1e-4 * rms))


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_sector_group_after_first_sector_removed(lower, name):
    """The group's first sector is removed (processor and plans destroyed) before another sector runs: the group
    launches with its own copy of the first plan, so the remaining sector's DL and UL still equal the reference."""
    check_group_sector(lower, CONFIGS[name], GROUP_FIRST_REMOVED)


@pytest.mark.parametrize("cfg", [CONFIG_60K_NORMAL, CONFIGS["60kHz_extended_cp"]], ids=["normal_cp", "extended_cp"])
def test_sector_group_mixed_cyclic_prefix(lower, cfg):
    """A 60 kHz sector joining a group whose first sector has the other cyclic prefix (same DFT size, bandwidth and
    slot length): a normal-CP slot has 14 jobs per port where the extended-CP first sector sized the group's job table
    for 12, so that sector must run alone; an extended-CP sector fits a normal-CP group. Both equal the reference."""
    check_group_sector(lower, cfg, GROUP_FIRST_OTHER_CP)
