#!/usr/bin/env python3
"""Lower-PHY processors (row b5) under a continuous slot script: the reference's own pdxch_processor_impl /
puxch_processor_impl (CPU OFDM objects, built from source by oracle/build_chain.sh) against the GPU processors of
integration/lower_phy_gpu.cpp, one sector, 100 MHz 30 kHz 4 ports. The DL script requests slot s + 2 before the lower
PHY processes every symbol of slot s (the radio unit's processing delay); the UL script requests slot s and delivers
its 14 symbols. Times the whole scenario call (the harness's per-symbol sample copies included for both variants) and
prints one JSON object; real time is 2 000 slots/s per sector.

--sectors S1,S2,...: the multi-sector sweep. S sectors share one GPU the way the reference's radio unit runs them
(one lower-PHY sector per cell, each driven by its own thread: lib/ru/generic/ru_factory_generic_impl.cpp:75-90): S
C++ threads (oracle/ref/ref_lower.cpp ref_lower_sectors_run) run the DL script together on their own processors, then
the UL script together; reported per S are the free-running aggregate slots/s and the slowest sector's slots/s,
then, paced at the radio's symbol rate from a common start, each direction's largest lag behind that pace (real time:
under one slot), for the reference CPU processors (host cores, up to --cpu-threads), the GPU processors one per
sector, and the GPU processors of one lower_phy_sector_group (one launch per symbol / slot for all sectors).
TEST INFRASTRUCTURE (diagnostic); GPU box:
    python tools/lower_phy_bench.py [--slots N] [--sectors 1,2,4,8,16]
"""
import argparse
import json
import resource
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests")]

import lower_harness as LH  # noqa: E402

CFG = dict(numerology=1, bw_rb=273, dft_size=4096, extended=False, center_freq_hz=3.5e9, nof_ports=4,
           window_offset=0.5)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", type=int, default=400)
    ap.add_argument("--grids", type=int, default=8)
    ap.add_argument("--sectors", default="", help="comma-separated sector counts for the multi-sector sweep")
    ap.add_argument("--window-us", type=int, default=0, help="sector group gather window (0: the group's defaults)")
    ap.add_argument("--cpu-threads", type=int, default=16, help="largest sector count for the reference CPU sweep")
    ap.add_argument("--sweep-only", default="", help="sweep only: comma list of cpu, gpu0, gpu4, gpu13, group0, "
                                                    "group4, group13 (default all, after the single-sector runs)")
    args = ap.parse_args()
    rng = np.random.default_rng(3)
    lower = LH.Lower()
    S, G, P, nsc = args.slots, args.grids, CFG["nof_ports"], 12 * CFG["bw_rb"]
    B = 100
    grids = (rng.integers(0, 1 << 16, (G, P, 14, nsc, 2))).astype(np.uint16)
    grids[..., 1] &= 0x3fff  # finite bf16 values
    grids[..., 0] &= 0x3fff
    mask = np.full(G, (1 << P) - 1, np.uint32)
    dl = [(LH.REQUEST, B + s, s % G, 0) for s in range(2)]
    for s in range(S):
        dl.append((LH.REQUEST, B + s + 2, (s + 2) % G, 0))
        dl.append((LH.PROCESS, B + s, 0, 14))
    ul = []
    for s in range(S):
        ul.append((LH.REQUEST, B + s, s % G, 0))
        ul.append((LH.PROCESS, B + s, 0, 14))
    n = sum(P * LH.symbol_size(CFG["numerology"], CFG["dft_size"], False, e[1], l)
            for e in ul if e[0] == LH.PROCESS for l in range(e[2], e[3]))
    samples = ((rng.normal(size=n) + 1j * rng.normal(size=n)) * 0.05).astype(np.complex64)
    out = {"config": dict(CFG, slots=S), "pdxch": {}, "puxch": {}}
    single = (("reference CPU processor", LH.REF_CPU), ("GPU processor", LH.GPU_PROCESSOR))
    for name, variant in () if args.sweep_only else single:
        lower.pdxch(variant, CFG, grids, mask, dl[:8])  # warm-up: plans, DFT tables
        t0 = time.perf_counter()
        _, flags, late = lower.pdxch(variant, CFG, grids, mask, dl)
        t = time.perf_counter() - t0
        out["pdxch"][name] = {"seconds": t, "slots_per_s": S / t, "late": len(late), "processed": int(flags.sum())}
        for inflight in ((2,) if variant == LH.REF_CPU else (2, 4, 7, 14)):
            key = name if variant == LH.REF_CPU else f"{name}, {inflight} symbols in flight"
            lower.puxch(variant, CFG, G, ul[:4], samples[: 2 * P * 14 * 5000], inflight)
            t0 = time.perf_counter()
            _, flags, rx, late = lower.puxch(variant, CFG, G, ul, samples, inflight)
            t = time.perf_counter() - t0
            out["puxch"][key] = {"seconds": t, "slots_per_s": S / t, "late": len(late), "notifications": len(rx)}
            print(json.dumps({key: out["puxch"][key]}), file=sys.stderr, flush=True)
    if args.sectors:
        out["sectors"] = sweep(lower, args, grids, mask, dl, ul, samples)
    print(json.dumps(out))


MAX_LAG = 0.5e-3  # a paced sector keeps real time while no symbol starts more than one slot behind its time
RING = 2 * 4 * 14 * (4096 + 352)  # DL baseband ring of the sweep: two slots of 4 ports (complex samples)


def sweep(lower, args, grids, mask, dl, ul, samples):
    """ref_lower_sectors_run: S sectors on their own C++ threads, all running the DL script together and then the UL
    script together; the sectors' carriers 20 MHz apart, each with its own copy of the grids and samples."""
    S, G = args.slots, args.grids
    res = {}
    runs = {"cpu": ("reference CPU processor", LH.REF_CPU, 0),
            "gpu0": ("GPU processor", LH.GPU_PROCESSOR, 0), "gpu4": ("GPU processor", LH.GPU_PROCESSOR, 4),
            "gpu13": ("GPU processor", LH.GPU_PROCESSOR, 13),
            "group0": ("GPU sector group", LH.GPU_GROUP, 0), "group4": ("GPU sector group", LH.GPU_GROUP, 4),
            "group13": ("GPU sector group", LH.GPU_GROUP, 13)}
    runs = [runs[k] for k in (args.sweep_only or "cpu,gpu0,gpu4,gpu13,group0,group4,group13").split(",")]
    for name, variant, inflight in runs:
        key = name if variant == LH.REF_CPU else f"{name}, {inflight} symbols in flight"
        res[key] = {}
        for nsec in (int(v) for v in args.sectors.split(",")):
            if variant == LH.REF_CPU and nsec > args.cpu_threads:
                continue
            freqs = [CFG["center_freq_hz"] + 2e7 * k for k in range(nsec)]
            g = np.broadcast_to(grids, (nsec,) + grids.shape)
            m = np.broadcast_to(mask, (nsec,) + mask.shape)
            x = samples  # one copy, read by every sector
            w = args.window_us
            lower.sectors(variant, CFG, freqs, g, m, dl[:8], ul[:4], x, inflight, ring=RING, window_us=w)  # warm-up
            r = lower.sectors(variant, CFG, freqs, g, m, dl, ul, x, inflight, ring=RING, window_us=w)
            sec = r["seconds"]
            # Paced: every sector at the radio's symbol rate from a common start. It keeps real
            # time when it ends less than a slot behind and under 1 % of its symbols started more than a slot late
            # (this host is no real-time system: a lone scheduling hiccup is forgiven, a growing lag is not).
            ru0, t0 = resource.getrusage(resource.RUSAGE_SELF), time.perf_counter()
            p = lower.sectors(variant, CFG, freqs, g, m, dl, ul, samples, inflight, ring=RING, window_us=w, paced=True)
            ru1, t1 = resource.getrusage(resource.RUSAGE_SELF), time.perf_counter()
            cpus = (ru1.ru_utime + ru1.ru_stime - ru0.ru_utime - ru0.ru_stime) / (t1 - t0)
            lag = p["lag"]
            res[key][str(nsec)] = {
                "free_running": {
                    "pdxch_slowest_sector_slots_per_s": S / sec[:, 0].max(),
                    "puxch_slowest_sector_slots_per_s": S / sec[:, 1].max(),
                    "pdxch_aggregate_slots_per_s": nsec * S / sec[:, 0].max(),
                    "puxch_aggregate_slots_per_s": nsec * S / sec[:, 1].max()},
                "paced_max_lag_us": {"pdxch": 1e6 * lag[:, 0].max(), "puxch": 1e6 * lag[:, 1].max()},
                "paced_final_lag_us": {"pdxch": 1e6 * lag[:, 2].max(), "puxch": 1e6 * lag[:, 3].max()},
                "paced_late_fraction": {"pdxch": lag[:, 4].max(), "puxch": lag[:, 5].max()},
                "paced_cpus_busy": cpus,
                "paced_longest_call_us": {"pdxch": 1e6 * lag[:, 6].max(), "puxch": 1e6 * lag[:, 7].max()},
                "paced_calls_over_a_symbol": {"pdxch": lag[:, 8].max(), "puxch": lag[:, 9].max()},
                "late": sum(len(v) for v in r["late"]) + sum(len(v) for v in p["late"]),
                "notifications": sum(len(u[2]) for u in p["ul"]),
                "real_time": bool(lag[:, 2:4].max() < MAX_LAG and lag[:, 4:6].max() < 0.01)}
            if variant == LH.GPU_GROUP:
                res[key][str(nsec)]["group_paced"] = p["group"]
            if variant == LH.GPU_GROUP:
                res[key][str(nsec)]["group"] = r["group"]
            print(json.dumps({key: {nsec: res[key][str(nsec)]}}), file=sys.stderr, flush=True)
        rt = [int(k) for k, v in res[key].items() if v["real_time"]]
        res[key]["sectors_at_real_time"] = max(rt) if rt else 0
    return res


if __name__ == "__main__":
    main()
