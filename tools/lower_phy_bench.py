#!/usr/bin/env python3
"""Lower-PHY processors (row b5) under a continuous slot script: the reference's own pdxch_processor_impl /
puxch_processor_impl (CPU OFDM objects, built from source by oracle/build_chain.sh) against the GPU processors of
integration/lower_phy_gpu.cpp, one sector, 100 MHz 30 kHz 4 ports. The DL script requests slot s + 2 before the lower
PHY processes every symbol of slot s (the radio unit's processing delay); the UL script requests slot s and delivers
its 14 symbols. Times the whole scenario call (the harness's per-symbol sample copies included for both variants) and
prints one JSON object; real time is 2 000 slots/s per sector. TEST INFRASTRUCTURE (diagnostic); GPU box:
    python tools/lower_phy_bench.py [--slots N]
"""
import argparse
import json
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
    ap.add_argument("--slots", type=int, default=200)
    ap.add_argument("--grids", type=int, default=8)
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
    for name, variant in (("reference CPU processor", LH.REF_CPU), ("GPU processor", LH.GPU_PROCESSOR)):
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
    print(json.dumps(out))


if __name__ == "__main__":
    main()
