#!/usr/bin/env python3
"""Benchmark: 100 MHz 4x4 PDSCH + PUSCH slot processing on MI355X (the whole upper-PHY data path plus OFDM).

BASELINE.json metric: "PDSCH+PUSCH slots/sec (100MHz 4x4) + LDPC info-bits/s at 1/2/4/8 GPU".
Workload ("n78 100 MHz 4x4, 273 PRB, LDPC BG1, batched 64 UEs"): one slot = 64 UEs sharing 273 PRBs (4-5 PRB each),
4 layers, 256QAM MCS 27 (table 2), one DM-RS symbol (type 1, 2 CDM groups without data) -> 64 transport blocks, 192
LDPC BG1 codeblocks (Z 288/352), 1.258 Mbit of TB payload per direction. A step processes `--slots-per-step` such
slots per GPU, both directions, on two HIP streams (as a gNB runs them concurrently):

  * DL: PDSCH encoder (TB CRC, segmentation, CB CRC, LDPC, rate matching) -> PDSCH DM-RS -> PDSCH modulator
    (scrambling, 256QAM, layer mapping, precoding, RE mapping, bf16 grid) -> OFDM modulator (4096-point DFT, CP,
    phase compensation) of 4 ports: baseband samples.
  * UL: OFDM demodulator of 4 rx ports -> DM-RS channel estimator (4 layers x 4 ports) -> PUSCH demodulator (4x4
    MMSE, soft demapping, descrambling) -> PUSCH decoder (rate dematching, LDPC min-sum, 6 iterations max with CRC
    early stop, SIMD arithmetic; TB CRC).
    Received samples: the UL transport blocks through a UE transmitter (the same GPU encoder / DM-RS / modulator),
    a per-UE random unitary 4x4 channel and AWGN (--snr-db), OFDM-modulated; synthesised once before timing and
    resident in HBM. `--worst-case` feeds Gaussian noise instead (no TB ever valid: every codeblock runs all
    iterations, like the reference ldpc_decoder_benchmark).

Weak scaling: every rank processes its own cells' slots; the decoded UL TBs + CRC flags of all ranks are gathered to
rank 0 (the FAPI rank) over RCCL once per step. One JSON line from rank 0.
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
from srsgpu import slot as slotlib  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
SLOT_RATE_30KHZ = 2000.0  # slots per second of one cell at 30 kHz SCS
DL_STAGES = ["pdsch_encode", "pdsch_dmrs_modulate", "ofdm_modulate"]
UL_STAGES = ["ofdm_demodulate", "pusch_channel_estimate", "pusch_demodulate", "pusch_decode"]


def cpu_baseline(ues, segs, tb_host, cw_host, llr_host, samples_host, iterations, budget_s):
    """The srsRAN reference built from its own sources (oracle/_ref) on ONE host core, same slot: PDSCH encoding of
    the 64 TBs (pdsch_encoder_impl: segmenter + AVX2 LDPC encoder + rate matcher), PDSCH DM-RS + modulation of the 64
    UEs into one grid and OFDM modulation of 4 ports (generic DFT), OFDM demodulation of 4 ports, per-UE DM-RS channel
    estimation + PUSCH demodulation (the open-source reference estimates / equalizes one layer: single-layer UEs on
    the same REs), and the PUSCH codeblock tasks of the 192 codeblocks (rate dematcher + LDPC decoder with CRC early
    stop, the implementations "auto" picks here)."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libsrsref.so")
    if not os.path.exists(ref_so):
        return None
    lib = ctypes.CDLL(ref_so)
    P = ctypes.c_void_p
    for f in ("ref_pdsch_encode_slot_timed", "ref_pusch_decode_cbs_timed", "ref_dl_slot_timed", "ref_ul_slot_timed"):
        getattr(lib, f).restype = ctypes.c_longlong
    avx512 = bool(lib.ref_cpu_has_avx512())
    vbmi = bool(lib.ref_cpu_has_avx512vbmi())
    n = len(ues)
    bg = np.array([s.base_graph for s in segs], np.int32)
    qm = np.array([u.qm for u in ues], np.int32)
    ly = np.array([u.nof_layers for u in ues], np.int32)
    ns = np.array([u.nof_ch_symbols for u in ues], np.uint32)
    tbb = np.array([s.tbs // 8 for s in segs], np.uint32)
    nrb = np.array([u.n_prb for u in ues], np.int32)
    rb0 = np.concatenate([[0], np.cumsum(nrb)[:-1]]).astype(np.int32)
    cw_off = np.array(cw_host[1], np.int32)
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
    t_enc = t_dec = t_dl = t_ul = t_dl_ofdm = t_ul_ofdm = t_chest = 0
    o1, o2 = ctypes.c_longlong(), ctypes.c_longlong()
    slots = 0
    t0 = time.time()
    while time.time() - t0 < budget_s or slots == 0:
        t_enc += lib.ref_pdsch_encode_slot_timed(1, n, bg.ctypes.data_as(P), qm.ctypes.data_as(P),
                                                 ly.ctypes.data_as(P), ns.ctypes.data_as(P), tbb.ctypes.data_as(P),
                                                 tb_host.ctypes.data_as(P), cw.ctypes.data_as(P))
        t_dl += lib.ref_dl_slot_timed(n, rb0.ctypes.data_as(P), nrb.ctypes.data_as(P), int(qm[0]), int(ly[0]),
                                      cw_host[0].ctypes.data_as(P), cw_off.ctypes.data_as(P), ctypes.byref(o1))
        t_dl_ofdm += o1.value
        t_ul += lib.ref_ul_slot_timed(n, rb0.ctypes.data_as(P), nrb.ctypes.data_as(P), int(qm[0]),
                                      samples_host.ctypes.data_as(P), ctypes.byref(o1), ctypes.byref(o2))
        t_ul_ofdm += o1.value
        t_chest += o2.value
        t_dec += lib.ref_pusch_decode_cbs_timed(2 if vbmi else 1, 2 if avx512 else 1, len(params),
                                                params.ctypes.data_as(P), llr_host.ctypes.data_as(P), iterations,
                                                iters.ctypes.data_as(P))
        slots += 1
    slot_s = (t_enc + t_dl + t_ul + t_dec) * 1e-9 / slots
    ms = lambda v: v * 1e-6 / slots  # noqa: E731
    return {"value": 1.0 / slot_s, "unit": "slots/s", "cores": 1, "kind": "reference",
            "sample": f"{slots} slots (64 UEs, 192 codeblocks per direction) through the srsRAN reference on one "
                      f"core: PDSCH encode {ms(t_enc):.2f} ms/slot (avx2 encoder), PDSCH DM-RS + modulation "
                      f"{ms(t_dl - t_dl_ofdm):.2f} + OFDM modulation {ms(t_dl_ofdm):.2f} ms/slot (generic DFT), OFDM "
                      f"demodulation {ms(t_ul_ofdm):.2f} + channel estimation {ms(t_chest):.2f} + PUSCH "
                      f"demodulation {ms(t_ul - t_ul_ofdm - t_chest):.2f} ms/slot (single-layer: the open-source "
                      f"reference's limit), PUSCH codeblock tasks {ms(t_dec):.2f} ms/slot "
                      f"({'avx512' if vbmi else 'avx2'} dematcher, {'avx512' if avx512 else 'avx2'} decoder, "
                      f"{iterations} iterations max, early stop, avg "
                      f"{np.where(iters > 0, iters, iterations).mean():.2f} iterations)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--slots-per-step", type=int, default=16)
    ap.add_argument("--iterations", type=int, default=6)
    ap.add_argument("--snr-db", type=float, default=35.0)
    ap.add_argument("--worst-case", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--serial-legs", action="store_true",
                    help="run the DL and UL legs on one stream (clean per-stage times; slower overall)")
    ap.add_argument("--batches", type=int, default=1,
                    help="split a step's slots into this many independent DL/UL pipeline pairs on their own streams")
    ap.add_argument("--graph", action=argparse.BooleanOptionalAction, default=True,
                    help="replay the DL+UL pipeline of a step as one captured HIP graph (default) or launch eagerly")
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
    B = args.batches
    assert B >= 1 and S % B == 0, "--slots-per-step must be a multiple of --batches"
    Sb = S // B  # slots per pipeline pair

    ues = sch.slot_100mhz_4x4()
    segs = [u.segmentation() for u in ues]
    cell = slotlib.CellSlots(ues, segs, Sb)
    dls = [slotlib.DownlinkPipeline(ctx, cell) for _ in range(B)]
    uls = [slotlib.UplinkPipeline(ctx, cell, iterations=args.iterations) for _ in range(B)]
    dl, ul = dls[0], uls[0]
    dl_tbs = [torch.randint(0, 256, (dl.tb_total,), generator=gen, device=dev, dtype=torch.uint8) for _ in range(B)]
    ul_tbs_tx = [torch.randint(0, 256, (dl.tb_total,), generator=gen, device=dev, dtype=torch.uint8) for _ in range(B)]
    if args.worst_case:
        samples = [torch.randn(2 * ul.ofdm.nof_samples, generator=gen, device=dev) * 0.01 for _ in range(B)]
        data_desc = "Gaussian noise samples (no TB ever valid: all LDPC iterations, worst case)"
    else:
        samples = [slotlib.synthesize_uplink(ctx, cell, ul_tbs_tx[b], snr_db=args.snr_db, seed=99 + rank + 1000 * b)
                   for b in range(B)]
        data_desc = (f"UL TBs through a GPU UE transmitter (same encoder / DM-RS / modulator), a random unitary 4x4 "
                     f"channel per UE and AWGN at {args.snr_db:g} dB SNR, OFDM-modulated (synthetic)")
    d_dl_tbs, d_ul_tbs_tx, d_samples = dl_tbs[0], ul_tbs_tx[0], samples[0]
    torch.cuda.synchronize()
    tb_bytes = dl.tb_bytes
    nof_tbs = len(tb_bytes)

    dl_streams = [torch.cuda.Stream(dev) for _ in range(B)]
    ul_streams = dl_streams if args.serial_legs else [torch.cuda.Stream(dev) for _ in range(B)]
    tb_gather = None
    if world > 1:
        from srsgpu import dist as sdist
        tb_gather = sdist.TbGather(ul.d_tbs.numel(), ul.d_tb_ok.numel(), dev, root=0)

    def pipeline(ev_dl=None, ev_ul=None, batches=None):
        """DL and UL legs of one step (every batch), forked from and joined back into the caller's current stream.
        Stage events, when given, go to batch 0."""
        cur = torch.cuda.current_stream(dev)
        bs = range(B) if batches is None else batches
        for b in bs:
            dl_streams[b].wait_stream(cur)
            ul_streams[b].wait_stream(cur)
        for b in bs:
            dls[b].execute(dl_tbs[b], dl_streams[b], ev_dl if b == 0 else None)
            uls[b].execute(samples[b], ul_streams[b], ev_ul if b == 0 else None)
        for b in bs:
            cur.wait_stream(dl_streams[b])
            cur.wait_stream(ul_streams[b])

    graph = None

    def step(ev_dl=None, ev_ul=None):
        if graph is not None and ev_dl is None:
            graph.replay()
        else:
            pipeline(ev_dl, ev_ul)
        if tb_gather is not None:
            for u in uls:
                tb_gather.gather(u.d_tbs, u.d_tb_ok)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    dl.encoder.stage_times()
    ul.decoder.stage_times()
    if args.graph:
        # hipGraph of the whole per-step pipeline (every plan is allocation-free and capture-safe): the 11 kernels,
        # the codeword memset and the stream fork/join replay as one graph launch per step.
        # thread_local: the RCCL watchdog thread of a multi-GPU run keeps polling its events during the capture.
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            pipeline()
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
    # Timed loop: eager mode records only the decoder plan's own stage events (the roofline kernel's launch duration,
    # on its launch stream); graph mode records none. The roofline kernel time then comes from an untimed eager pass
    # with those two events, and per-stage times from another untimed pass with events between the stages.
    ul.decoder.enable_timing(not args.graph, decode_only=True)
    evs = [([torch.cuda.Event(enable_timing=True) for _ in range(4)],
            [torch.cuda.Event(enable_timing=True) for _ in range(5)]) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if args.graph:
        ul.decoder.enable_timing(True, decode_only=True)
        for _ in range(args.steps):
            pipeline(batches=[0])  # the roofline kernel of batch 0, its pipeline pair alone
        torch.cuda.synchronize()
    ul_ms, ul_n = ul.decoder.stage_times()
    assert ul_n == args.steps
    ul.decoder.enable_timing(False)
    for i in range(args.steps):  # per-stage times: an extra, untimed pass of batch 0 with events between the stages
        pipeline(*evs[i], batches=[0])
    torch.cuda.synchronize()
    stage = {k: 0.0 for k in DL_STAGES + UL_STAGES}
    for ed, eu in evs:
        for j, k in enumerate(DL_STAGES):
            stage[k] += ed[j].elapsed_time(ed[j + 1]) / args.steps
        for j, k in enumerate(UL_STAGES):
            stage[k] += eu[j].elapsed_time(eu[j + 1]) / args.steps
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    # ---- Results of the last step: UL TB success (decoded TBs must equal what the UEs sent) and iterations ----
    tb_ok = np.concatenate([u.d_tb_ok.cpu().numpy().astype(bool) for u in uls])
    iters = np.concatenate([u.d_iters.cpu().numpy() for u in uls])
    if not args.worst_case:
        for b in range(B):
            sent = ul_tbs_tx[b].cpu().numpy()
            got = uls[b].d_tbs.cpu().numpy()
            ok_b = uls[b].d_tb_ok.cpu().numpy().astype(bool)
            off = 0
            for i, nb in enumerate(tb_bytes):
                if ok_b[i]:
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
    dec_bytes = ul.decoder.decoder_input_llrs + sum(
        s.nof_segments * (((22 if s.base_graph == 1 else 10) * s.lifting_size + 7) // 8 + 45) for s in segs) * Sb
    achieved = dec_bytes / (dec_ms * 1e-3) / 1e9
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "ldpc_decode_traffic.json")
    if os.path.exists(tfile):
        with open(tfile) as f:
            tj = json.load(f)
        if tj.get("slots_per_step") == Sb and tj.get("worst_case", False) == args.worst_case:
            traffic = tj.get("hbm_bytes_per_launch")

    # VALU roofline of the same launch: wave-level VALU instructions per launch from the committed SQ counter pass
    # (rocprofv3 --pmc SQ_INSTS_VALU ..., tools/sq_summary.py; same workload, same iterations) over the live kernel time.
    valu = None
    sqfile = os.path.join(ROOT, "profiles", "r1_v22_sq_valu.json")
    if os.path.exists(sqfile) and Sb == 16 and not args.worst_case:
        with open(sqfile) as f:
            sq = json.load(f).get("ldpc_decode_pk_kernel<1, 1, 8>")
        if sq:
            peak = 1024 * 2.4e9 / 2  # SIMDs x clock / 2 cycles per wave64 VALU instruction (MI355X_MICROARCH.md)
            rate = sq["valu_instr"] / (dec_ms * 1e-3)
            valu = {"bound": "valu_issue", "achieved": rate, "peak": peak, "unit": "wave-instr/s",
                    "frac": rate / peak, "instr_per_launch": sq["valu_instr"],
                    "source": "profiles/r1_v22_sq_valu.json (SQ_INSTS_VALU) / live kernel time"}

    # Algorithmic HBM bytes per pipeline pair (Sb slots) of the signal-chain stages (each byte read or written once;
    # DESIGN.md "Kernels"): bf16 grids are 4 B per RE, time samples 8 B (complex float), estimates 4 B per (layer,
    # port, RE), LLRs 1 B. The stage times come from batch 0's pipeline pair.
    S_all, S = S, Sb
    P, nsc, L = cell.nof_ports, cell.nsc, ues[0].nof_layers
    grid_b = S * P * 14 * nsc * 4
    spp = ul.ofdm.nof_samples // (S * P)  # samples per slot and port (CPs included)
    data_re = S * sum(12 * u.n_prb * (14 - 1) for u in ues)  # one DM-RS symbol without data
    cw_b = sum(s.cw_length for s in segs) * S // 8
    ce_rows = 1 if ul.estimate_layout == srsgpu.CE_COMPACT else 14  # estimate rows per (layer, port) and slot
    ce_b = S * L * P * ce_rows * nsc * 4
    stage_bytes = {
        "pdsch_dmrs_modulate": cw_b + grid_b,
        "ofdm_modulate": grid_b + S * P * spp * 8,
        "ofdm_demodulate": S * P * 14 * slotlib.DFT_SIZE * 8 + grid_b,
        "pusch_channel_estimate": S * P * nsc * 4 + ce_b,
        "pusch_demodulate": data_re * (P * 4 + L * ues[0].qm) + ce_b,
    }
    stage_gbps = {k: v / (stage[k] * 1e-3) / 1e9 for k, v in stage_bytes.items() if stage[k] > 0}

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
        "dtype": "int8/bf16/f32",
        "data": "synthetic: random TB payloads; PUSCH input = " + data_desc,
        "config": {"workload": "n78 100 MHz 4x4 slot, 273 PRB, 64 UEs x (4-5 PRB, 4 layers, 256QAM MCS27), LDPC BG1 "
                               "(Z 288/352): 64 TBs / 192 codeblocks per direction per slot",
                   "dl_chain": "PDSCH encoder -> PDSCH DM-RS -> PDSCH modulator -> OFDM modulator (4 ports)",
                   "ul_chain": "OFDM demodulator (4 ports) -> DM-RS channel estimator (4 layers x 4 ports) -> PUSCH "
                               "demodulator (MMSE 4x4) -> PUSCH decoder",
                   "channel_estimate_layout": "compact (one row per allocation, average time strategy)"
                                              if ul.estimate_layout == srsgpu.CE_COMPACT else "per symbol",
                   "leg_streams": "one stream" if args.serial_legs else "DL and UL on concurrent streams",
                   "launch": "one captured HIP graph per step (torch.cuda.CUDAGraph over the plans' execute calls)"
                             if args.graph else "eager kernel launches",
                   "slots_per_step": S_all,
                   "concurrent_batches": f"{B} DL/UL pipeline pair(s) of {Sb} slots, each leg on its own stream",
                   "codeblocks_per_step_per_direction": int(sum(s.nof_segments for s in segs) * S_all),
                   "ldpc_max_iterations": args.iterations, "ldpc_early_stop": True,
                   "decoder_arithmetic": "avx2/avx512 (SIMD) variant, bit-exact",
                   "ofdm": "4096-point DFT, 122.88 Msps, normal CP",
                   "parallelism": (f"dp{world}: each GPU processes its own cells' slots; decoded UL TBs + CRC flags "
                                   f"gathered to the FAPI rank over RCCL every step") if world > 1 else
                                  "dp1 (independent cells per GPU)"},
        "ldpc_info_bits_per_s": info_bits_slot * value,
        "tb_bits_per_s_per_direction": tbs_bits_slot * value,
        "realtime_cells_per_gpu": value / SLOT_RATE_30KHZ / world,
        "pusch_tb_success_rate": float(tb_ok.mean()),
        "ldpc_avg_iterations": avg_iters,
        "stage_ms_per_step": stage,  # from the untimed pass of batch 0 with per-stage events
        "stage_slots": Sb,
        "stage_algorithmic_gbps": stage_gbps,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": "ldpc_decode_pk_kernel<1,1,8>",
                     "kernel_ms_per_launch": dec_ms,
                     "note": "algorithmic bytes per launch / decoder-stage HIP-event time on the launch stream ("
                             + ("an eager pass of as many steps right after the graph-replayed timed loop"
                                if args.graph else "inside the timed loop")
                             + "); the LDPC decoder is VALU-issue/latency-bound, not HBM-bound (DESIGN.md)"},
        "roofline_valu": valu,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        n_slot = len(segs)
        tb_host = d_dl_tbs[: sum(tb_bytes[:n_slot])].cpu().numpy()
        cw_host = (dl.d_cw.cpu().numpy(), dl.cw_offsets[:n_slot])
        llr_host = ul.d_llrs[: sum(s.cw_length for s in segs)].cpu().numpy()
        samples_host = d_samples[: 2 * 4 * 61440].cpu().numpy()
        result["cpu_baseline"] = cpu_baseline(ues, segs, tb_host, cw_host, llr_host, samples_host, args.iterations,
                                              args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
