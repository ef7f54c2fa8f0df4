"""GPU parity of the OFDM slot modulator / demodulator (srsgpu_ofdm_plan through the C ABI) against the reference's
own outputs (tests/golden/ofdm.npz, made by ofdm_slot_modulator_impl / ofdm_slot_demodulator_impl with the generic
DFT) and the complex128 restatement (oracle/ofdm_oracle.py).

Tolerances (floating point, stated here as the north star asks): modulated samples within 2e-5 x RMS of the
reference / oracle (the reference's own float DFT sits at ~1e-6); demodulated bf16 grids: every value within one bf16
ulp (<= 2^-7 relative) or 1e-4 x RMS absolute, and < 2 % of the significant values differing at all (rounding-boundary
cases of the float DFT)."""
import numpy as np
import pytest

import golden_lib as G
import ofdm_oracle as O
from ofdm_cases import CASES, bf16_close, random_grid, rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import srsgpu
    return srsgpu.Context(0)


def test_ofdm_golden(ctx):
    import srsgpu
    n = 0
    for (mu, rb, N, ext, scale, fc, slot, woff), grid, samples, demod in G.ofdm_cases():
        mod = srsgpu.OfdmSlotModulator(ctx, mu, rb, N, scale, fc, cp_extended=ext)
        got = mod.modulate(grid, slot)
        assert got.shape == samples.shape
        assert rel_err(got, samples) < 2e-5
        dem = srsgpu.OfdmSlotDemodulator(ctx, mu, rb, N, 1.0 / (scale * N), fc, cp_extended=ext, window_offset=woff)
        g2 = dem.demodulate(samples, slot)
        ok, frac = bf16_close(g2, demod)
        assert ok and frac < 0.02, frac
        n += 1
    assert n == 5


@pytest.mark.parametrize("case", range(len(CASES)))
def test_ofdm_vs_oracle(ctx, case):
    import srsgpu
    mu, rb, N, ext, scale, fc, slot, woff = CASES[case]
    rng = np.random.default_rng(200 + case)
    ns = 12 if ext else 14
    grid = random_grid(rng, 2, ns, 12 * rb, occupancy=0.8)
    want = O.modulate(grid, mu, rb, N, ext, scale, fc, slot)
    got = srsgpu.OfdmSlotModulator(ctx, mu, rb, N, scale, fc, cp_extended=ext).modulate(grid, slot)
    assert rel_err(got, want) < 2e-5
    # Demodulate noisy samples (not a round trip: every bin carries energy).
    x = want + (rng.normal(size=want.shape) + 1j * rng.normal(size=want.shape)) * 0.01 * np.sqrt(
        np.mean(np.abs(want) ** 2))
    x = x.astype(np.complex64)
    gw = O.complex_to_bf16(O.demodulate(x.astype(np.complex128), mu, rb, N, ext, 0.37, fc, slot, woff))
    gg = srsgpu.OfdmSlotDemodulator(ctx, mu, rb, N, 0.37, fc, cp_extended=ext, window_offset=woff).demodulate(x, slot)
    ok, frac = bf16_close(gg, gw)
    assert ok and frac < 0.02, frac


def test_ofdm_batched_slots_round_trip(ctx):
    """The bench layout: 16 slots x 4 ports of 100 MHz grids in ONE plan each way (slots alternate between the two
    slots of the subframe). Modulation matches the oracle per (grid, port); demodulating the modulator's own output
    with scale 1 / (scale N) returns the input grid (bf16 round trip)."""
    import torch
    import srsgpu
    mu, rb, N, scale, fc = 1, 273, 4096, 1.0 / 64, 3.5e9
    rng = np.random.default_rng(7)
    S, P = 16, 4
    grids = random_grid(rng, S * P, 14, 12 * rb).reshape(S, P, 14, 12 * rb, 2)
    slots = [s % 2 for s in range(S)]
    dev = torch.device("cuda", 0)
    mod = srsgpu.OfdmPlan(ctx, True, mu, rb, N, scale, fc, slots, P)
    dem = srsgpu.OfdmPlan(ctx, False, mu, rb, N, 1.0 / (scale * N), fc, slots, P)
    assert mod.nof_samples == S * P * 61440
    d_grid = torch.from_numpy(grids.view(np.int32).reshape(-1).copy()).to(dev)
    d_x = torch.zeros(2 * mod.nof_samples, dtype=torch.float32, device=dev)
    d_back = torch.zeros_like(d_grid)
    mod.execute(d_grid, d_x)
    dem.execute(d_x, d_back)
    torch.cuda.synchronize()
    x = d_x.cpu().numpy().view(np.complex64)
    for s in (0, 1, 9):
        want = O.modulate(grids[s], mu, rb, N, False, scale, fc, slots[s])
        for p in range(P):
            o = mod.sample_offset(s, p)
            assert rel_err(x[o:o + 61440], want[p]) < 2e-5, (s, p)
    back = d_back.cpu().numpy().view(np.uint16).reshape(grids.shape)
    ok, frac = bf16_close(back, grids)
    assert ok and frac < 0.02, frac


def test_ofdm_rejects_invalid(ctx):
    import srsgpu
    for args in [(1, 273, 3000, 1.0, 0.0), (1, 273, 2048, 1.0, 0.0), (1, 106, 2048, 0.0, 0.0), (5, 10, 512, 1.0, 0.0),
                 (1, 273, 16384, 1.0, 0.0), (1, 273, 10000, 1.0, 0.0), (0, 5, 64, 1.0, 0.0)]:
        with pytest.raises(srsgpu.SrsGpuError):
            srsgpu.OfdmPlan(ctx, True, *args, [0], 1)
    with pytest.raises(srsgpu.SrsGpuError):  # window offset >= 144 N / 2048
        srsgpu.OfdmPlan(ctx, False, 1, 106, 2048, 1.0, 0.0, [0], 1, window_offset=144)
    with pytest.raises(srsgpu.SrsGpuError):  # slot index beyond the subframe
        srsgpu.OfdmPlan(ctx, True, 1, 106, 2048, 1.0, 0.0, [2], 1)


@pytest.mark.parametrize("inverse", [False, True])
def test_ofdm_plan_concat_sector_group(ctx, inverse):
    """srsgpu_ofdm_plan_concat (the lower-PHY sector group): three sectors with their own carrier frequency, scaling
    and symbol position in one plan give, bit for bit, what each sector's own plan gives on its slice of the grids and
    time samples; members that disagree on the launch-wide parameters are refused."""
    import torch
    import srsgpu
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(31)
    P = 2
    members = [srsgpu.OfdmPlan(ctx, inverse, 1, 106, 2048, sc, fc, [slot], P, window_offset=0 if inverse else 40,
                               symbols=(l, 1))
               for sc, fc, slot, l in ((0.5, 3.5e9, 0, 0), (0.25, 3.6e9, 1, 7), (1.0, 1.8e9, 1, 13))]
    group = srsgpu.OfdmPlan.concat(members)
    assert group.grid_words == sum(m.grid_words for m in members)
    assert group.nof_samples == sum(m.nof_samples for m in members)
    words = np.cumsum([0] + [m.grid_words for m in members])
    samples = np.cumsum([0] + [m.nof_samples for m in members])
    for i, m in enumerate(members):
        for p in range(P):
            assert group.sample_offset(i, p) == samples[i] + m.sample_offset(0, p)
    grids = rng.integers(0, 1 << 14, 2 * group.grid_words).astype(np.uint16).view(np.int32)
    x = (rng.normal(size=2 * group.nof_samples) * 0.1).astype(np.float32)
    src = torch.from_numpy(grids.copy() if inverse else x.copy()).to(dev)
    out = (torch.zeros(2 * group.nof_samples, dtype=torch.float32, device=dev) if inverse
           else torch.zeros(group.grid_words, dtype=torch.int32, device=dev))
    group.execute(src, out)
    for i, m in enumerate(members):
        if inverse:
            s_in = src[words[i]:words[i + 1]].clone()
            o = torch.zeros(2 * m.nof_samples, dtype=torch.float32, device=dev)
            m.execute(s_in, o)
            assert torch.equal(o, out[2 * samples[i]:2 * samples[i + 1]]), i
        else:
            s_in = src[2 * samples[i]:2 * samples[i + 1]].clone()
            o = torch.zeros(m.grid_words, dtype=torch.int32, device=dev)
            m.execute(s_in, o)
            assert torch.equal(o, out[words[i]:words[i + 1]]), i
    odd = srsgpu.OfdmPlan(ctx, inverse, 1, 52, 2048, 1.0, 3.5e9, [0], P, symbols=(0, 1))
    with pytest.raises(srsgpu.SrsGpuError):
        srsgpu.OfdmPlan.concat([members[0], odd])


@pytest.mark.parametrize("inverse", [False, True])
def test_ofdm_job_list_equals_plans(ctx, inverse):
    """srsgpu_ofdm_jobs_execute (the lower-PHY sector group's launch): the jobs of three sectors' plans (own carrier,
    scaling, slot and symbol), reordered and placed at offsets of the caller's choosing in one buffer pair, give bit for
    bit what each plan gives on its own buffers; a split DFT size is refused."""
    import torch
    import srsgpu
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(37)
    P = 2
    members = [srsgpu.OfdmPlan(ctx, inverse, 1, 106, 2048, sc, fc, [slot], P, window_offset=0 if inverse else 40,
                               symbols=(l, 1))
               for sc, fc, slot, l in ((0.5, 3.5e9, 0, 0), (0.25, 3.6e9, 1, 7), (1.0, 1.8e9, 1, 13))]
    # Member i's buffers sit at (word_base[i], sample_base[i]) of the shared buffers, in reverse order with gaps.
    word_base = [3 * 4096 + 7, 1 * 4096 + 5, 0 + 3][:3]
    sample_base = [9000 * 2 + 11, 9000 + 13, 17]
    jobs = []
    for i, m in enumerate(members):
        j = m.jobs()
        assert len(j) == P
        j["grid_offset"] += word_base[i]
        j["sample_offset"] += sample_base[i]
        jobs.append(j)
    jobs = np.concatenate(jobs)[::-1].copy()  # any order
    words, samples = 5 * 4096, 4 * 9000
    d_jobs = torch.from_numpy(jobs.view(np.uint8).copy()).to(dev)
    if inverse:
        src = torch.from_numpy(rng.integers(0, 1 << 14, 2 * words).astype(np.uint16).view(np.int32).copy()).to(dev)
        out = torch.zeros(2 * samples, dtype=torch.float32, device=dev)
    else:
        src = torch.from_numpy((rng.normal(size=2 * samples) * 0.1).astype(np.float32)).to(dev)
        out = torch.zeros(words, dtype=torch.int32, device=dev)
    members[0].execute_jobs(d_jobs, len(jobs), src, out)
    for i, m in enumerate(members):
        if inverse:
            o = torch.zeros(2 * m.nof_samples, dtype=torch.float32, device=dev)
            m.execute(src[word_base[i]:word_base[i] + m.grid_words].clone(), o)
            assert torch.equal(o, out[2 * sample_base[i]:2 * (sample_base[i] + m.nof_samples)]), i
        else:
            o = torch.zeros(m.grid_words, dtype=torch.int32, device=dev)
            m.execute(src[2 * sample_base[i]:2 * (sample_base[i] + m.nof_samples)].clone(), o)
            assert torch.equal(o, out[word_base[i]:word_base[i] + m.grid_words]), i
    split = srsgpu.OfdmPlan(ctx, inverse, 1, 273, 12288, 1.0, 3.5e9, [0], 1, symbols=(0, 1))
    with pytest.raises(srsgpu.SrsGpuError):
        split.execute_jobs(d_jobs, 1, src, out)


@pytest.mark.parametrize("inverse", [False, True])
def test_ofdm_direct_jobs_equal_plans(ctx, inverse):
    """srsgpu_ofdm_jobs_execute_direct (the sector group writing straight into a mapped uplink grid): three sectors'
    jobs with absolute addresses into three separate allocations per side, in any order, give bit for bit what each
    plan gives on its own buffers; a split DFT size is refused."""
    import torch
    import srsgpu
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(41)
    P = 2
    members = [srsgpu.OfdmPlan(ctx, inverse, 1, 106, 2048, sc, fc, [slot], P, window_offset=0 if inverse else 40,
                               symbols=(l, 1))
               for sc, fc, slot, l in ((0.5, 3.5e9, 0, 0), (0.25, 3.6e9, 1, 7), (1.0, 1.8e9, 1, 13))]
    grids, samples, jobs = [], [], []
    for m in members:
        g = torch.from_numpy(rng.integers(0, 1 << 14, 2 * m.grid_words).astype(np.uint16).view(np.int32).copy())
        x = torch.from_numpy((rng.normal(size=2 * m.nof_samples) * 0.1).astype(np.float32))
        grids.append((g if inverse else torch.zeros(m.grid_words, dtype=torch.int32)).to(dev))
        samples.append((torch.zeros(2 * m.nof_samples, dtype=torch.float32) if inverse else x).to(dev))
        jobs.append(m.direct_jobs(grids[-1], samples[-1]))
    # Demodulation: the second member's rows also go to a copy (grid_copy: the HBM twin of a mapped uplink grid).
    twin = torch.zeros(members[1].grid_words, dtype=torch.int32, device=dev)
    if not inverse:
        jobs[1]["grid_copy"] = jobs[1]["grid"] - np.uint64(srsgpu._dptr(grids[1])) + np.uint64(srsgpu._dptr(twin))
    jobs = np.concatenate(jobs)[::-1].copy()
    d_jobs = torch.from_numpy(jobs.view(np.uint8).copy()).to(dev)
    members[0].execute_jobs_direct(d_jobs, len(jobs))
    torch.cuda.synchronize()
    for i, m in enumerate(members):
        if inverse:
            o = torch.zeros(2 * m.nof_samples, dtype=torch.float32, device=dev)
            m.execute(grids[i], o)
            assert torch.equal(o, samples[i]), i
        else:
            o = torch.zeros(m.grid_words, dtype=torch.int32, device=dev)
            m.execute(samples[i], o)
            assert torch.equal(o, grids[i]), i
    if not inverse:
        assert torch.equal(twin, grids[1])
    split = srsgpu.OfdmPlan(ctx, inverse, 1, 273, 12288, 1.0, 3.5e9, [0], 1, symbols=(0, 1))
    with pytest.raises(srsgpu.SrsGpuError):
        split.execute_jobs_direct(d_jobs, 1)
