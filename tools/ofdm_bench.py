#!/usr/bin/env python3
"""Isolated OFDM modulator / demodulator launch time on the headline bench's shape (32 slots x 4 ports, 273 PRB,
4096-point DFT, normal CP): each plan executed back to back on one stream, HIP events around the loop; algorithmic
bytes per launch as bench.py counts them (grid 4 B per RE + 8 B per time sample, each once).

    python tools/ofdm_bench.py [--slots 32] [--iters 200]   (srsgpu from SRSGPU_LIB or the in-tree build)
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "srsran-5g_amd"))
import srsgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", type=int, default=32)
    ap.add_argument("--ports", type=int, default=4)
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    ctx = srsgpu.Context(0)
    dev = torch.device("cuda", 0)
    slots = [s % 2 for s in range(a.slots)]  # slot index within the subframe
    res = {"slots": a.slots, "ports": a.ports, "lib": os.environ.get("SRSGPU_LIB", "in-tree")}
    mod = srsgpu.OfdmPlan(ctx, True, 1, 273, 4096, 0.01, 3.5e9, slots, a.ports)
    dem = srsgpu.OfdmPlan(ctx, False, 1, 273, 4096, 1.0 / 4096, 3.5e9, slots, a.ports)
    rng = np.random.default_rng(1)
    grid = torch.from_numpy(rng.integers(0, 2 ** 31, mod.grid_words, dtype=np.int64).astype(np.int32)).to(dev)
    grid &= 0x3fff3fff  # finite bf16 pairs
    samples = torch.zeros(2 * mod.nof_samples, dtype=torch.float32, device=dev)
    grid_out = torch.zeros(dem.grid_words, dtype=torch.int32, device=dev)
    for name, plan, src, dst in (("ofdm_modulate", mod, grid, samples), ("ofdm_demodulate", dem, samples, grid_out)):
        for _ in range(10):
            plan.execute(src, dst)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            plan.execute(src, dst)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        alg = plan.grid_words * 4 + plan.nof_samples * 8
        res[name] = {"us_per_launch": us, "algorithmic_bytes": alg, "tb_per_s": alg / us / 1e6,
                     "hbm_fraction_8tbs": alg / us / 1e6 / 8.0}
        print(f"{name:16s} {us:7.2f} us  {alg / 1e6:6.1f} MB  {alg / us / 1e6:5.2f} TB/s  "
              f"{alg / us / 1e6 / 8.0:.3f} of 8 TB/s", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
