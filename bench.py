#!/usr/bin/env python3
"""Benchmark: 100 MHz 4x4 PDSCH + PUSCH channel-coding slot processing on MI355X.

BASELINE.json metric: "PDSCH+PUSCH slots/sec (100MHz 4x4) + LDPC info-bits/s at 1/2/4/8 GPU".
Workload ("n78 100 MHz 4x4, 273 PRB, LDPC BG1, batched 64 UEs"): one slot = 64 UEs sharing 273 PRBs (4-5 PRB each),
4 layers, 256QAM MCS 27 (table 2), one DM-RS symbol -> 64 transport blocks, 192 LDPC BG1 codeblocks (Z 288/352),
1.258 Mbit of TB payload per direction. A step processes `--slots-per-step` such slots per GPU, both directions:

  * PDSCH (DL): srsgpu_pdsch_encoder_plan — TB CRC, segmentation, CB CRC24B, LDPC encoding, rate matching.
  * PUSCH (UL): srsgpu_pusch_decoder_plan — rate dematching (new data), LDPC decoding (layered min-sum, SIMD
    arithmetic, `--iterations` max with CRC early stop; srsRAN default 6), CB concatenation, TB CRC24A.
    Received LLRs: the UL transport blocks encoded on the GPU, mapped to +/-amp with AWGN (--llr-amp/--llr-noise),
    synthesised once before timing and resident in HBM; `--worst-case` uses random +/-10 LLRs instead (never
    CRC-valid: every codeblock runs all iterations, like the reference ldpc_decoder_benchmark).

Weak scaling: every rank processes its own cells' slots; no data-path collective. One JSON line from rank 0.
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

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
SLOT_RATE_30KHZ = 2000.0  # slots per second of one cell at 30 kHz SCS


def slot_grants():
    ues = sch.slot_100mhz_4x4()
    return ues, [u.segmentation() for u in ues]


def synth_llrs(cw, cw_offsets, Gs, amp, noise, gen, dev):
    """Codeword bits (packed, per-TB word-aligned) -> int8 LLRs (contiguous G per TB): +/-amp + N(0, noise)."""
    idx = torch.cat([torch.arange(G, device=dev, dtype=torch.int64) + off * 8 for off, G in zip(cw_offsets, Gs)])
    byte = cw[idx >> 3].to(torch.int32)
    bits = (byte >> (7 - (idx & 7).to(torch.int32))) & 1
    llr = (1 - 2 * bits).to(torch.float32) * amp
    if noise > 0:
        llr = llr + torch.randn(llr.shape, generator=gen, device=dev) * noise
    return torch.clamp(torch.round(llr), -120, 120).to(torch.int8)


def cpu_baseline(ues, segs, tb_host, llr_host, iterations, budget_s):
    """The srsRAN reference built from its own sources (oracle/_ref) on ONE host core, same slot: PDSCH encoding of
    the 64 TBs (pdsch_encoder_impl: segmenter + AVX2 LDPC encoder + rate matcher) and the PUSCH codeblock tasks of the
    192 codeblocks (rate dematcher + LDPC decoder with CRC early stop, the implementations "auto" picks here)."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libsrsref.so")
    if not os.path.exists(ref_so):
        return None
    lib = ctypes.CDLL(ref_so)
    P = ctypes.c_void_p
    lib.ref_pdsch_encode_slot_timed.restype = ctypes.c_longlong
    lib.ref_pusch_decode_cbs_timed.restype = ctypes.c_longlong
    avx512 = bool(lib.ref_cpu_has_avx512())
    vbmi = bool(lib.ref_cpu_has_avx512vbmi())
    n = len(ues)
    bg = np.array([s.base_graph for s in segs], np.int32)
    qm = np.array([u.qm for u in ues], np.int32)
    ly = np.array([u.nof_layers for u in ues], np.int32)
    ns = np.array([u.nof_ch_symbols for u in ues], np.uint32)
    tbb = np.array([s.tbs // 8 for s in segs], np.uint32)
    cw = np.zeros(sum(s.cw_length for s in segs), np.uint8)
    params = []
    llr_off = 0
    for u, s in zip(ues, segs):
        crc = 1 if s.nof_segments > 1 else (0 if s.tbs > 3824 else 3)
        for cb in s.codeblocks:
            params.append([s.base_graph, s.lifting_size, u.qm, cb.rm_length, cb.nof_filler_bits, crc,
                           cb.nof_crc_bits, llr_off + cb.cw_offset])
        llr_off += s.cw_length
    params = np.array(params, np.int32)
    iters = np.zeros(len(params), np.int32)
    enc_ns = dec_ns = 0
    slots = 0
    t0 = time.time()
    while time.time() - t0 < budget_s or slots == 0:
        enc_ns += lib.ref_pdsch_encode_slot_timed(1, n, bg.ctypes.data_as(P), qm.ctypes.data_as(P),
                                                  ly.ctypes.data_as(P), ns.ctypes.data_as(P), tbb.ctypes.data_as(P),
                                                  tb_host.ctypes.data_as(P), cw.ctypes.data_as(P))
        dec_ns += lib.ref_pusch_decode_cbs_timed(2 if vbmi else 1, 2 if avx512 else 1, len(params),
                                                 params.ctypes.data_as(P), llr_host.ctypes.data_as(P), iterations,
                                                 iters.ctypes.data_as(P))
        slots += 1
    slot_s = (enc_ns + dec_ns) * 1e-9 / slots
    return {"value": 1.0 / slot_s, "unit": "slots/s", "cores": 1, "kind": "reference",
            "sample": f"{slots} slots (64 TBs + 192 codeblocks each) through the srsRAN reference on one core: PDSCH "
                      f"encode {enc_ns * 1e-6 / slots:.2f} ms/slot (avx2 encoder), PUSCH codeblock tasks "
                      f"{dec_ns * 1e-6 / slots:.2f} ms/slot ({'avx512' if vbmi else 'avx2'} dematcher, "
                      f"{'avx512' if avx512 else 'avx2'} decoder, {iterations} iterations max, early stop, avg "
                      f"{np.where(iters > 0, iters, iterations).mean():.2f} iterations)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--slots-per-step", type=int, default=16)
    ap.add_argument("--iterations", type=int, default=6)
    ap.add_argument("--llr-amp", type=float, default=16.0)
    ap.add_argument("--llr-noise", type=float, default=6.0)
    ap.add_argument("--worst-case", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--serial-legs", action="store_true",
                    help="run the DL and UL legs on one stream (clean per-stage times; slower overall)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    ctx = srsgpu.Context(local_rank)
    S = args.slots_per_step

    ues, segs = slot_grants()
    tb_bytes = [s.tbs // 8 for s in segs] * S
    Gs = [s.cw_length for s in segs] * S
    nof_tbs = len(tb_bytes)

    # ---- PDSCH leg ----
    dl_cfgs = [srsgpu.PdschTransportBlock(s.base_graph, 0, u.qm, u.nof_layers, u.nof_ch_symbols)
               for u, s in zip(ues, segs)] * S
    dl_arr, dl_tb_total, dl_cw_total, dl_cw_offsets = srsgpu.make_pdsch_configs(tb_bytes, dl_cfgs)
    dl_plan = srsgpu.PdschEncoderPlan(ctx, dl_arr)
    d_dl_tbs = torch.randint(0, 256, (dl_tb_total,), generator=gen, device=dev, dtype=torch.uint8)
    d_dl_cw = torch.zeros(dl_cw_total, dtype=torch.uint8, device=dev)

    # ---- PUSCH leg: received LLRs of GPU-encoded UL transport blocks ----
    d_ul_tbs_tx = torch.randint(0, 256, (dl_tb_total,), generator=gen, device=dev, dtype=torch.uint8)
    d_ul_cw = torch.zeros(dl_cw_total, dtype=torch.uint8, device=dev)
    enc_tmp = srsgpu.PdschEncoderPlan(ctx, dl_arr)
    enc_tmp.execute(d_ul_tbs_tx, d_ul_cw)
    if args.worst_case:
        d_llrs = (torch.randint(0, 2, (sum(Gs),), generator=gen, device=dev, dtype=torch.int32) * 20 - 10).to(torch.int8)
        data_desc = "random +/-10 LLRs (never CRC-valid: all iterations, worst case)"
    else:
        d_llrs = synth_llrs(d_ul_cw, dl_cw_offsets, Gs, args.llr_amp, args.llr_noise, gen, dev)
        data_desc = (f"UL TBs encoded on the GPU, BPSK-mapped to +/-{args.llr_amp:g} LLRs + AWGN sigma "
                     f"{args.llr_noise:g} (synthetic)")
    torch.cuda.synchronize()
    enc_tmp.close()
    ul_cfgs = [srsgpu.PuschTransportBlock(s.tbs // 8, s.base_graph, 0, u.qm, u.nof_layers, u.nof_ch_symbols,
                                          nof_ldpc_iterations=args.iterations) for u, s in zip(ues, segs)] * S
    nof_cbs = [s.nof_segments for s in segs] * S
    cb_len = [(66 if s.base_graph == 1 else 50) * s.lifting_size for s in segs] * S
    ul_arr, ul_llr_total, harq_total, cb_total, ul_tb_total = srsgpu.make_pusch_tb_configs(ul_cfgs, nof_cbs, cb_len)
    ul_plan = srsgpu.PuschDecoderPlan(ctx, srsgpu.IMPL_SIMD, ul_arr)
    d_harq = torch.zeros(harq_total, dtype=torch.int8, device=dev)
    d_crc = torch.zeros(cb_total, dtype=torch.uint8, device=dev)
    d_msgs = torch.zeros(cb_total * srsgpu.CB_MSG_STRIDE, dtype=torch.uint8, device=dev)
    d_iters = torch.zeros(cb_total, dtype=torch.int32, device=dev)
    d_ul_tbs = torch.zeros(ul_tb_total, dtype=torch.uint8, device=dev)
    d_tb_ok = torch.zeros(nof_tbs, dtype=torch.uint8, device=dev)
    # The DL and UL legs are independent (as in a gNB, where PDSCH and PUSCH processing of a slot run concurrently):
    # each gets its own HIP stream, joined back into the main stream at the end of every step.
    main_stream = torch.cuda.current_stream(dev)
    dl_stream = torch.cuda.Stream(dev)
    ul_stream = dl_stream if args.serial_legs else torch.cuda.Stream(dev)

    # Multi-GPU (north star): every rank codes its own cells' slots; the decoded UL transport blocks and their CRC flags
    # of all ranks are gathered to the FAPI rank (rank 0) over RCCL once per step - the path's only exchange.
    tb_gather = None
    if world > 1:
        from srsgpu import dist as sdist
        tb_gather = sdist.TbGather(d_ul_tbs.numel(), d_tb_ok.numel(), dev, root=0)

    def step():
        dl_stream.wait_stream(main_stream)
        ul_stream.wait_stream(main_stream)
        dl_plan.execute(d_dl_tbs, d_dl_cw, dl_stream)
        ul_plan.execute(d_llrs, d_harq, d_crc, d_msgs, d_iters, d_ul_tbs, d_tb_ok, ul_stream)
        main_stream.wait_stream(dl_stream)
        main_stream.wait_stream(ul_stream)
        if tb_gather is not None:
            tb_gather.gather(d_ul_tbs, d_tb_ok)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    dl_plan.stage_times()
    ul_plan.stage_times()
    dl_plan.enable_timing(True)
    ul_plan.enable_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    dl_ms, dl_n = dl_plan.stage_times()
    ul_ms, ul_n = ul_plan.stage_times()
    assert dl_n == args.steps and ul_n == args.steps
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    # ---- Results of the last step: UL TB success and iterations (decoded TBs must equal what was sent) ----
    tb_ok = d_tb_ok.cpu().numpy().astype(bool)
    iters = d_iters.cpu().numpy()
    if not args.worst_case:
        sent = d_ul_tbs_tx.cpu().numpy()
        got = d_ul_tbs.cpu().numpy()
        off = 0
        for i, nb in enumerate(tb_bytes):
            if tb_ok[i]:
                assert np.array_equal(got[off:off + nb], sent[off:off + nb]), f"TB {i} CRC ok but payload differs"
            off += nb
    avg_iters = float(np.where(iters > 0, iters, args.iterations).mean())

    slots = S * world * args.steps
    value = slots / elapsed
    info_bits_slot = sum(((22 if s.base_graph == 1 else 10) * s.lifting_size - s.nof_filler_bits) * s.nof_segments
                         for s in segs)
    tbs_bits_slot = sum(s.tbs for s in segs)
    dec_ms = ul_ms[1] / args.steps
    # Algorithmic bytes of one decoder launch: the LLRs each codeblock's decode() reads (the HARQ span up to the
    # dematcher's zero tail, as reported by the plan), K*Z/8 bytes of decoded bits written, 4 B result + 1 B CRC flag,
    # 40 B descriptor.
    dec_bytes = ul_plan.decoder_input_llrs + sum(
        s.nof_segments * (((22 if s.base_graph == 1 else 10) * s.lifting_size + 7) // 8 + 45) for s in segs) * S
    achieved = dec_bytes / (dec_ms * 1e-3) / 1e9
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "ldpc_decode_traffic.json")
    if os.path.exists(tfile):
        with open(tfile) as f:
            tj = json.load(f)
        if tj.get("slots_per_step") == S and tj.get("worst_case", False) == args.worst_case:
            traffic = tj.get("hbm_bytes_per_launch")

    result = {
        "metric": "PDSCH+PUSCH slots/sec (100MHz 4x4) + LDPC info-bits/s at 1/2/4/8 GPU",
        "value": value,
        "unit": "slots/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8",
        "data": "synthetic: random TB payloads; PUSCH LLRs = " + data_desc,
        "config": {"workload": "n78 100 MHz 4x4 slot, 273 PRB, 64 UEs x (4-5 PRB, 4 layers, 256QAM MCS27), LDPC BG1 "
                               "(Z 288/352): 64 TBs / 192 codeblocks per direction per slot",
                   "legs": ["pdsch_encode", "pusch_decode"],
                   "leg_streams": "one stream" if args.serial_legs else "DL and UL on concurrent streams",
                   "slots_per_step": S,
                   "codeblocks_per_step_per_direction": int(sum(nof_cbs)),
                   "ldpc_max_iterations": args.iterations, "ldpc_early_stop": True,
                   "decoder_arithmetic": "avx2/avx512 (SIMD) variant, bit-exact",
                   "parallelism": (f"dp{world}: each GPU codes its own cells' slots; decoded UL TBs + CRC flags "
                                   f"gathered to the FAPI rank over RCCL every step") if world > 1 else
                                  "dp1 (independent cells per GPU)"},
        "ldpc_info_bits_per_s": info_bits_slot * value,
        "tb_bits_per_s_per_direction": tbs_bits_slot * value,
        "realtime_cells_per_gpu": value / SLOT_RATE_30KHZ / world,
        "pusch_tb_success_rate": float(tb_ok.mean()),
        "ldpc_avg_iterations": avg_iters,
        "stage_ms_per_step": {"pdsch_tb_crc": dl_ms[0] / args.steps, "pdsch_encode_rm": dl_ms[1] / args.steps,
                              "pusch_rate_dematch": ul_ms[0] / args.steps, "pusch_ldpc_decode": dec_ms,
                              "pusch_tb_crc": ul_ms[2] / args.steps},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": "ldpc_decode_pk_kernel<1,1,8>",
                     "kernel_ms_per_launch": dec_ms,
                     "note": "algorithmic bytes per launch / decoder-stage HIP-event time on the launch stream; the "
                             "LDPC decoder is VALU-issue/latency-bound, not HBM-bound (DESIGN.md)"},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # One slot's UL payloads and LLRs on the host (same data the GPU decodes).
        n_slot = len(segs)
        tb_host = d_dl_tbs[: sum(tb_bytes[:n_slot])].cpu().numpy()
        llr_host = d_llrs[: sum(Gs[:n_slot])].cpu().numpy()
        result["cpu_baseline"] = cpu_baseline(ues, segs, tb_host, llr_host, args.iterations, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
