#!/usr/bin/env python3
"""Benchmark: 100 MHz 4x4 slot processing on MI355X (BASELINE.json metric "PDSCH+PUSCH slots/sec (100MHz 4x4) + LDPC
info-bits/s at 1/2/4/8 GPU").

Workload (config "n78 100 MHz 4x4, 273 PRB, LDPC BG1, batched 64 UEs"): one slot = 64 UEs sharing 273 PRBs, 4 layers,
256QAM MCS 27 (table 2), one DM-RS symbol -> 192 LDPC BG1 codeblocks (Z 288/352), 1.258 Mbit of transport blocks.
A step processes `--slots-per-step` such slots on every GPU (weak scaling: each rank owns its own cells' slots; no
data-path collective). Legs timed inside a step:
  * pusch_ldpc_decode: the PUSCH decoder's LDPC stage over the rate-dematched codeblock buffers (8 iterations max,
    CRC24B early stop). Inputs are synthetic random +/-10 LLRs (the reference benchmark's input,
    tests/benchmarks/phy/upper/channel_coding/ldpc/ldpc_decoder_benchmark.cpp:129), which never pass the CRC: every
    codeblock runs all 8 iterations (worst case).

Run: python bench.py [--gpus N --steps K --warmup W]; N>1 under torch.distributed.run (one rank per GPU, RCCL).
Rank 0 prints ONE JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "srsran-5g_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import srsgpu  # noqa: E402
from srsgpu import sch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def build_slot(rng, nof_ues=64):
    """Per-codeblock decoder configs and rate-dematched LLR buffers of one 100 MHz 4x4 slot."""
    ues = sch.slot_100mhz_4x4(nof_ues)
    cbs = []
    tbs_bits = 0
    for ue in ues:
        seg = ue.segmentation()
        tbs_bits += seg.tbs
        K = 22 if seg.base_graph == 1 else 10
        N = (66 if seg.base_graph == 1 else 50) * seg.lifting_size
        nsys = (K - 2) * seg.lifting_size
        for cb in seg.codeblocks:
            # rv 0, new data: LLRs land on [0, nsys - F) and [nsys, ...) (ldpc_rate_dematcher_impl.cpp:128); filler
            # positions are +inf; the rest of the circular buffer stays zero.
            buf = np.zeros(N, np.int8)
            info = nsys - cb.nof_filler_bits
            n_par = cb.rm_length - info
            buf[:info] = (rng.integers(0, 2, info) * 20 - 10).astype(np.int8)
            buf[info:nsys] = 127
            buf[nsys:nsys + n_par] = (rng.integers(0, 2, n_par) * 20 - 10).astype(np.int8)
            cbs.append(dict(bg=seg.base_graph, Z=seg.lifting_size, filler=cb.nof_filler_bits,
                            crc_bits=cb.nof_crc_bits, crc_poly=srsgpu.CRC24B if seg.nof_segments > 1 else
                            (srsgpu.CRC24A if seg.tbs > 3824 else srsgpu.CRC16), llr=buf,
                            info_bits=K * seg.lifting_size - cb.nof_filler_bits))
    return cbs, tbs_bits


def cpu_baseline(cbs, max_iter, budget_s):
    """The srsRAN reference decoder (built from its own sources, oracle/_ref) on one host core, over a bounded sample
    of the same codeblocks. Implementation: AVX-512 if the host has it, else AVX2 — what create_ldpc_decoder_factory_sw
    ("auto") picks."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libsrsref.so")
    if not os.path.exists(ref_so):
        return None
    lib = ctypes.CDLL(ref_so)
    lib.ref_ldpc_decode_timed.restype = ctypes.c_longlong
    lib.ref_ldpc_decode_timed.argtypes = [ctypes.c_int] * 7 + [ctypes.c_float, ctypes.c_void_p, ctypes.c_uint,
                                                                ctypes.c_uint, ctypes.c_uint, ctypes.c_void_p]
    impl = 2 if lib.ref_cpu_has_avx512() else 1
    total_ns = 0
    n_done = 0
    t_start = time.time()
    i = 0
    while time.time() - t_start < budget_s:
        c = cbs[i % len(cbs)]
        it = np.zeros(1, np.int32)
        total_ns += lib.ref_ldpc_decode_timed(impl, c["bg"], c["Z"], c["crc_bits"], c["filler"], c["crc_poly"],
                                              max_iter, ctypes.c_float(0.8), c["llr"].ctypes.data, c["llr"].size,
                                              c["llr"].size, 1, it.ctypes.data)
        n_done += 1
        i += 1
    per_cb_s = total_ns * 1e-9 / n_done
    slot_s = per_cb_s * len(cbs)
    return {"value": 1.0 / slot_s, "unit": "slots/s", "cores": 1, "kind": "reference",
            "sample": f"{n_done} codeblocks of the slot (BG1 Z 288/352, {max_iter} iterations) decoded by the srsRAN "
                      f"{'avx512' if impl == 2 else 'avx2'} LDPC decoder on one core, {total_ns * 1e-9:.1f} s; "
                      f"scaled to the slot's {len(cbs)} codeblocks"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--slots-per-step", type=int, default=16)
    ap.add_argument("--iterations", type=int, default=8)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    rng = np.random.default_rng(1234 + rank)
    slot_cbs, slot_tbs_bits = build_slot(rng)
    S = args.slots_per_step
    ctx = srsgpu.Context(local_rank)

    # ---- PUSCH LDPC decode leg: S slots x 192 codeblocks, one plan, inputs resident in HBM. ----
    cfgs = []
    llr_host = []
    polys = []
    for s in range(S):
        for c in slot_cbs:
            cfgs.append(srsgpu.CodeblockDecodeConfig(c["bg"], c["Z"], nof_crc_bits=c["crc_bits"],
                                                     nof_filler_bits=c["filler"], max_iterations=args.iterations))
            llr_host.append(c["llr"])
            polys.append(c["crc_poly"])
    nof_llrs = [x.size for x in llr_host]
    arr = srsgpu.make_configs(cfgs, nof_llrs, polys)
    plan = srsgpu.LdpcDecoderPlan(ctx, srsgpu.IMPL_SIMD, arr)
    d_llrs = torch.from_numpy(np.concatenate(llr_host)).to(dev)
    out_bytes = sum((srsgpu.BG_K[c.base_graph] * c.lifting_size + 7) // 8 for c in cfgs)
    d_out = torch.zeros(out_bytes, dtype=torch.uint8, device=dev)
    d_iters = torch.zeros(len(cfgs), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        plan.execute(d_llrs, d_out, d_iters, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps  # one decoder launch per step (single base graph)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    iters = d_iters.cpu().numpy()
    assert (iters == -1).all(), "random LLRs must never pass the CRC (worst-case workload)"

    slots = S * world * args.steps
    value = slots / elapsed
    ms_per_step = elapsed * 1e3 / args.steps
    info_bits_slot = sum(c["info_bits"] for c in slot_cbs)
    alg_bytes = sum(nof_llrs) + out_bytes + 4 * len(cfgs) + 40 * len(cfgs)
    achieved_gbs = alg_bytes / (kernel_ms * 1e-3) / 1e9
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "ldpc_decode_traffic.json")
    if os.path.exists(tfile):
        with open(tfile) as f:
            tj = json.load(f)
        if tj.get("slots_per_step") == S:
            traffic = tj.get("hbm_bytes_per_launch")

    result = {
        "metric": "PDSCH+PUSCH slots/sec (100MHz 4x4) + LDPC info-bits/s at 1/2/4/8 GPU",
        "value": value,
        "unit": "slots/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8",
        "data": "synthetic: random +/-10 LLRs (reference ldpc_decoder_benchmark input), never CRC-valid -> all "
                f"{args.iterations} iterations run (worst case)",
        "config": {"workload": "n78 100 MHz 4x4, 273 PRB, 64 UEs, MCS27 256QAM, LDPC BG1 (Z 288/352), "
                               "192 codeblocks per slot",
                   "legs": ["pusch_ldpc_decode"], "slots_per_step": S, "codeblocks_per_step": len(cfgs),
                   "ldpc_max_iterations": args.iterations, "decoder_arithmetic": "avx2/avx512 (SIMD) variant",
                   "parallelism": f"dp{world} (codeblocks of independent cells per GPU, no collective)"},
        "ldpc_info_bits_per_s": info_bits_slot * value,
        "tb_bits_per_s": slot_tbs_bits * value,
        "realtime_factor_30khz": value / 2000.0 / world,
        "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "ldpc_decode_kernel<1,1>", "kernel_ms": kernel_ms,
                     "note": "algorithmic bytes = LLRs in + packed bits out + results + descriptors; the decoder is "
                             "VALU/LDS-bound (8 iterations x edges per codeblock), see DESIGN.md"},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(slot_cbs, args.iterations, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
