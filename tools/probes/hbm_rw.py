#!/usr/bin/env python3
"""HBM read / write / copy rates on this GPU with torch's own kernels (the ceilings the OFDM kernels are judged
against): write-only fill, read-only sum, and a copy, each over a buffer far larger than the 256 MB Infinity Cache.

    python tools/probes/hbm_rw.py [--mb 1024] [--iters 20]
"""
import argparse
import json

import torch


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    n = a.mb * (1 << 20) // 4
    x = torch.empty(n, dtype=torch.float32, device="cuda")
    y = torch.empty(n, dtype=torch.float32, device="cuda")
    x.fill_(1.0)
    out = {}
    b = n * 4
    t = timed(lambda: x.fill_(2.0), a.iters)
    out["write_tb_s"] = b / t / 1e12
    t = timed(lambda: x.sum(), a.iters)
    out["read_tb_s"] = b / t / 1e12
    t = timed(lambda: y.copy_(x), a.iters)
    out["copy_tb_s"] = 2 * b / t / 1e12
    out["buffer_mb"] = a.mb
    print(json.dumps(out))


if __name__ == "__main__":
    main()
