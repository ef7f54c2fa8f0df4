#!/usr/bin/env python3
"""Decoder kernel time vs iterations (no CRC: every codeblock runs max_iterations) for the bench's codeblock shapes,
plain vs edge-split kernel (SRSGPU_OPTION_DECODER_SPLIT, read at plan creation): fixed cost + per-iteration cost.

    python tools/decoder_sweep.py [--n 1024] [--z 224] [--cols 27]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "srsran-5g_amd"))

import torch  # noqa: E402

import srsgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[1024, 3072])
    ap.add_argument("--z", type=int, default=224)
    ap.add_argument("--cols", type=int, default=27, help="input span in lifted columns (rate-matched E / Z + 2)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = srsgpu.Context(0)
    Z = args.z
    n_llr = (args.cols - 2) * Z
    rng = np.random.default_rng(3)
    llr1 = np.clip(np.round(16.0 + rng.normal(0, 6.0, n_llr)), -120, 120).astype(np.int8)
    for n in args.n:
        for split in ("0", "1"):
            ctx.set_option(srsgpu.OPTION_DECODER_SPLIT, int(split))
            row = []
            for iters in range(1, 7):
                cfg = srsgpu.CodeblockDecodeConfig(1, Z, nof_crc_bits=16, max_iterations=iters)
                arr = srsgpu.make_configs([cfg] * n, [n_llr] * n, [srsgpu.CRC_NONE] * n)
                plan = srsgpu.LdpcDecoderPlan(ctx, srsgpu.IMPL_SIMD, arr)
                d_llr = torch.from_numpy(np.tile(llr1, n)).to(dev)
                d_out = torch.zeros(n * ((22 * Z + 7) // 8), dtype=torch.uint8, device=dev)
                d_it = torch.zeros(n, dtype=torch.int32, device=dev)
                for _ in range(3):
                    plan.execute(d_llr, d_out, d_it)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                reps = 20
                e0.record()
                for _ in range(reps):
                    plan.execute(d_llr, d_out, d_it)
                e1.record()
                torch.cuda.synchronize()
                row.append(e0.elapsed_time(e1) / reps * 1e3)
                plan.close()
            slope = np.polyfit(np.arange(1, 7), row, 1)
            print(f"n={n:5d} Z={Z} split={split}: " + " ".join(f"{t:6.1f}" for t in row) +
                  f" us  (fixed {slope[1]:.1f} + {slope[0]:.1f} us/iteration)", flush=True)


if __name__ == "__main__":
    main()
