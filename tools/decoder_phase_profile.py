#!/usr/bin/env python3
"""Phase breakdown of the LDPC decoder kernel on the bench workload (instrumented build).

Build the instrumented library first (it goes next to, not over, the product library):
    SRSGPU_OUT_DIR=srsran-5g_amd/lib_prof SRSGPU_EXTRA_FLAGS=-DLDPC_DEC_PROFILE bash srsran-5g_amd/build.sh
then run on the GPU:
    SRSGPU_LIB=srsran-5g_amd/lib_prof/libsrsgpu_phy.so python tools/decoder_phase_profile.py [--worst-case]

Each codeblock's workgroup stamps s_memtime at: start (0), after the LLR load (1), after the layers of iteration k
(2+2k) and after its CRC check (3+2k), after the output (28); s_memrealtime (100 MHz) at start/end (29/30) and the
number of layers (31). Prints per-phase average cycles and the kernel-wide concurrency picture.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "srsran-5g_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import srsgpu  # noqa: E402

SLOTS = 32


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", type=int, default=16)
    ap.add_argument("--iterations", type=int, default=6)
    ap.add_argument("--worst-case", action="store_true")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234)
    ctx = srsgpu.Context(0)
    lib = srsgpu.load_library()
    if not hasattr(lib, "srsgpu_debug_decoder_profile"):
        raise SystemExit("not an instrumented build (set SRSGPU_LIB to the LDPC_DEC_PROFILE library)")
    S = args.slots
    ues, segs = bench.slot_grants()
    tb_bytes = [s.tbs // 8 for s in segs] * S
    Gs = [s.cw_length for s in segs] * S
    cfgs = [srsgpu.PdschTransportBlock(s.base_graph, 0, u.qm, u.nof_layers, u.nof_ch_symbols)
            for u, s in zip(ues, segs)] * S
    arr, tb_total, cw_total, cw_offsets = srsgpu.make_pdsch_configs(tb_bytes, cfgs)
    tbs = torch.randint(0, 256, (tb_total,), generator=gen, device=dev, dtype=torch.uint8)
    cw = torch.zeros(cw_total, dtype=torch.uint8, device=dev)
    enc = srsgpu.PdschEncoderPlan(ctx, arr)
    enc.execute(tbs, cw)
    if args.worst_case:
        llrs = (torch.randint(0, 2, (sum(Gs),), generator=gen, device=dev, dtype=torch.int32) * 20 - 10).to(torch.int8)
    else:
        llrs = bench.synth_llrs(cw, cw_offsets, Gs, 16.0, 6.0, gen, dev)
    ul_cfgs = [srsgpu.PuschTransportBlock(s.tbs // 8, s.base_graph, 0, u.qm, u.nof_layers, u.nof_ch_symbols,
                                          nof_ldpc_iterations=args.iterations) for u, s in zip(ues, segs)] * S
    nof_cbs = [s.nof_segments for s in segs] * S
    cb_len = [(66 if s.base_graph == 1 else 50) * s.lifting_size for s in segs] * S
    ul_arr, llr_total, harq_total, cb_total, ul_tb_total = srsgpu.make_pusch_tb_configs(ul_cfgs, nof_cbs, cb_len)
    plan = srsgpu.PuschDecoderPlan(ctx, srsgpu.IMPL_SIMD, ul_arr)
    harq = torch.zeros(harq_total, dtype=torch.int8, device=dev)
    crc = torch.zeros(cb_total, dtype=torch.uint8, device=dev)
    msgs = torch.zeros(cb_total * srsgpu.CB_MSG_STRIDE, dtype=torch.uint8, device=dev)
    iters = torch.zeros(cb_total, dtype=torch.int32, device=dev)
    out_tbs = torch.zeros(ul_tb_total, dtype=torch.uint8, device=dev)
    tb_ok = torch.zeros(len(tb_bytes), dtype=torch.uint8, device=dev)
    for _ in range(3):
        plan.execute(llrs, harq, crc, msgs, iters, out_tbs, tb_ok)
    torch.cuda.synchronize()

    n = min(cb_total, 4096)
    buf = np.zeros(n * SLOTS, dtype=np.uint64)
    lib.srsgpu_debug_decoder_profile.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]
    # Even lifting sizes run on the packed kernel (its own stamp array); fall back to the one-row kernel's.
    assert lib.srsgpu_debug_decoder_profile(buf.ctypes.data, buf.size, 1) == 0
    if not buf.any():
        assert lib.srsgpu_debug_decoder_profile(buf.ctypes.data, buf.size, 0) == 0
    p = buf.reshape(n, SLOTS).astype(np.int64)
    it = iters.cpu().numpy()[:n]
    # Keep codeblocks whose stamps all come from the last launch (a codeblock that returned early keeps stale ones).
    nit0 = np.where(it > 0, it, args.iterations)
    ok = (p[:, 30] > p[:, 29]) & (p[:, 1] >= p[:, 0]) & (p[:, 28] >= p[:, 1])
    for k in range(args.iterations):
        ok &= ~(nit0 > k) | ((p[:, 2 + 2 * k] >= p[:, 1]) & (p[:, 3 + 2 * k] >= p[:, 2 + 2 * k]))
    p, it = p[ok], it[ok]
    n = int(ok.sum())
    nit = np.where(it > 0, it, args.iterations)
    t0 = p[:, 0]
    res = {"nof_cbs": int(n), "avg_iterations": float(nit.mean()), "nof_layers": np.bincount(p[:, 31]).tolist()}
    res["load_cycles"] = float((p[:, 1] - t0).mean())
    lay, crcc = [], []
    for k in range(int(nit.max())):
        sel = nit > k
        prev = p[sel, 1] if k == 0 else p[sel, 3 + 2 * (k - 1)]
        lay.append(float((p[sel, 2 + 2 * k] - prev).mean()))
        crcc.append(float((p[sel, 3 + 2 * k] - p[sel, 2 + 2 * k]).mean()))
    res["layers_cycles_per_iteration"] = lay
    res["crc_cycles_per_iteration"] = crcc
    last = np.array([p[i, 3 + 2 * (nit[i] - 1)] for i in range(n)])
    res["output_cycles"] = float((p[:, 28] - last).mean())
    res["total_cycles_per_cb"] = float((p[:, 28] - t0).mean())
    wall = (p[:, 30] - p[:, 29]) / 100.0  # us
    res["cb_wall_us_avg"] = float(wall.mean())
    res["kernel_span_us"] = float((p[:, 30].max() - p[:, 29].min()) / 100.0)
    res["clock_ghz_est"] = float(((p[:, 28] - t0) / np.maximum(wall, 1e-3) / 1e3).mean())
    # Concurrency: average number of codeblocks resident at once.
    res["avg_resident_cbs"] = float(wall.sum() / max(res["kernel_span_us"], 1e-9))
    # Iteration-0 layer time by start-time quartile (first resident round vs later codeblocks).
    start = p[:, 29]
    q = np.quantile(start, [0.25, 0.5, 0.75])
    it0 = (p[:, 2] - p[:, 1]).astype(float)
    grp = np.searchsorted(q, start)
    res["iter0_cycles_by_start_quartile"] = [float(it0[grp == g].mean()) for g in range(4)]
    it1 = np.where(nit > 1, (p[:, 4] - p[:, 3]).astype(float), np.nan)
    res["iter1_cycles_by_start_quartile"] = [float(np.nanmean(it1[grp == g])) for g in range(4)]
    load = (p[:, 1] - p[:, 0]).astype(float)
    res["load_cycles_by_start_quartile"] = [float(load[grp == g].mean()) for g in range(4)]
    # Residency timeline: codeblocks in flight per 10 us bin, and how many start / finish in each bin.
    t_lo = p[:, 29].min()
    st = (p[:, 29] - t_lo) / 100.0
    en = (p[:, 30] - t_lo) / 100.0
    bins = np.arange(0.0, en.max() + 10.0, 10.0)
    res["timeline_us"] = [float(b) for b in bins[:-1]]
    res["timeline_resident"] = [int(((st < b + 10) & (en > b)).sum()) for b in bins[:-1]]
    res["timeline_starts"] = np.histogram(st, bins)[0].tolist()
    res["timeline_ends"] = np.histogram(en, bins)[0].tolist()
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
