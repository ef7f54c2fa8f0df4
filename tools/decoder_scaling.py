#!/usr/bin/env python3
"""Decoder throughput vs batch size: the same codeblock (BG1, Z = 288, high-rate 4-layer span, noisy LLRs from the
oracle-free encoder path) decoded N times in one plan, N = 256 .. 8192. Prints kernel time per launch (HIP events)
and codeblocks per microsecond, i.e. how throughput scales with the number of codeblocks in flight.

    python tools/decoder_scaling.py [--iters 6] [--z 288] [--cols 26]
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
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--z", type=int, default=288)
    ap.add_argument("--cols", type=int, default=26, help="input span in lifted columns (K + 4 = 26: 4 layers)")
    ap.add_argument("--noise", type=float, default=6.0)
    ap.add_argument("--no-crc", action="store_true")
    ap.add_argument("--sizes", default="256,512,1024,2048,3072,4096,8192", help="codeblocks per launch")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = srsgpu.Context(0)
    Z = args.z
    n_llr = (args.cols - 2) * Z
    rng = np.random.default_rng(3)
    # All-zero codeword (valid for any LDPC code): +amp LLRs with noise. With CRC16 the all-zero message passes.
    llr1 = np.clip(np.round(16.0 + rng.normal(0, args.noise, n_llr)), -120, 120).astype(np.int8)
    for n in [int(x) for x in args.sizes.split(",")]:
        cfg = srsgpu.CodeblockDecodeConfig(1, Z, nof_crc_bits=16, max_iterations=args.iters)
        polys = [srsgpu.CRC_NONE if args.no_crc else srsgpu.CRC16] * n
        arr = srsgpu.make_configs([cfg] * n, [n_llr] * n, polys)
        plan = srsgpu.LdpcDecoderPlan(ctx, srsgpu.IMPL_SIMD, arr)
        d_llr = torch.from_numpy(np.tile(llr1, n)).to(dev)
        d_out = torch.zeros(n * ((22 * Z + 7) // 8), dtype=torch.uint8, device=dev)
        d_it = torch.zeros(n, dtype=torch.int32, device=dev)
        for _ in range(3):
            plan.execute(d_llr, d_out, d_it)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            plan.execute(d_llr, d_out, d_it)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        it = d_it.cpu().numpy()
        print(f"n={n:5d}  {ms * 1e3:8.1f} us/launch  {n / (ms * 1e3):6.2f} cb/us  iterations {np.unique(it)}",
              flush=True)
        plan.close()


if __name__ == "__main__":
    main()
