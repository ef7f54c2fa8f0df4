#!/usr/bin/env python3
"""The reference's PHY processor benchmarks (pusch_processor_benchmark.cpp, pdsch_processor_benchmark.cpp, "throughput
total" mode) restated over the reference's own processors (oracle/_ref/libsrschain.so: pusch_processor_impl /
pdsch_processor_impl built from their sources) on the reference's CPU components and on the GPU bindings of
integration/ (the benchmarks themselves cannot be built here: the reference's DFT factories need FFTW, absent from
this image). Same profiles, PDUs, thread / batch / repetition scheme; prints one JSON object.

GPU box: python tools/processor_bench.py [--threads N] [--batch B] [--repetitions R] > out.json
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "srsran-5g_amd")]

import chain_harness as H  # noqa: E402
from srsgpu import sch  # noqa: E402


def host_cores():
    n = len(os.sched_getaffinity(0))
    cap = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(cap))) if cap and cap.isdigit() else n


def run(lib, fn, mode, p, tbs, threads, batch, reps, weights=None):
    import ctypes
    secs = np.zeros(reps, np.float64)
    args = [0, mode, ctypes.byref(p)]
    if weights is not None:
        w = np.ascontiguousarray(weights, np.complex64).view(np.float32)
        args.append(w.ctypes.data_as(ctypes.c_void_p))
    args += [tbs // 8, threads, batch, reps, secs.ctypes.data_as(ctypes.c_void_p)]
    r = fn(*args)
    assert r >= 0, f"benchmark failed ({r})"
    pdus = threads * batch
    med = float(np.median(secs))
    return {"mode": mode, "threads": threads, "batch_per_thread": batch, "repetitions": reps,
            "seconds_median": med, "throughput_mbps_median": pdus * tbs / med / 1e6,
            "throughput_mbps_max": pdus * tbs / float(np.min(secs)) / 1e6,
            "pdus_per_s": pdus / med, "tb_crc_ok": int(r)}


def slot_cases(lib, T, slots, R, directions=("ul", "dl"), pace_us=0.0):
    """The same profiles through the reference's slot processors (uplink_processor_impl /
    downlink_processor_single_executor_impl), one per thread, reference CPU processors (variant 0) vs the GPU slot batches
    of integration/pusch_batch_gpu.cpp / upper_phy_gpu.cpp (variant 1: one synchronous uplink processor per thread;
    UL variant 2: du_low's shape - a ring of uplink processors per sector, asynchronous completion, one GPU service
    gathering every sector's slot into one launch): the single full-band PDU per slot of the reference benchmarks, and the
    multi-UE slot at the slot processors' capacity (MAX_PUSCH_PDUS_PER_SLOT = MAX_UE_PDUS_PER_SLOT = 16,
    slot_pdu_capacity_constants.h:44/:77: 16 UEs x 17 PRB) where the batch gathers the 16 PDUs into one launch
    sequence."""
    import ctypes
    PP = ctypes.POINTER(H.ChainParams)
    lib.chain_ul_bench.restype = ctypes.c_int
    lib.chain_ul_bench.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint,
                                   ctypes.c_int, PP, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint, ctypes.c_uint,
                                   ctypes.c_void_p, ctypes.c_double, ctypes.c_void_p]
    lib.chain_dl_bench.restype = ctypes.c_int
    lib.chain_dl_bench.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint,
                                   ctypes.c_int, PP, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint,
                                   ctypes.c_uint, ctypes.c_void_p]
    rng = np.random.default_rng(1)
    out = {"ul": [], "dl": []}
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731

    def ul(name, pdus, tbs):
        arr = (H.ChainParams * len(pdus))(*pdus)
        tbb = np.array(tbs, np.int32) // 8
        grid = (rng.normal(size=(4, 14, 12 * 273, 2)) * 0.1).astype(np.float32)
        g = ((grid.view(np.uint32) + 0x7FFF + ((grid.view(np.uint32) >> 16) & 1)) >> 16).astype(np.uint16)
        case = {"profile": name, "nof_pdus_per_slot": len(pdus), "tb_bits_per_slot": int(sum(tbs)), "runs": []}
        for v in (0, 1, 2):
            n = slots
            secs = np.zeros(R, np.float64)
            lat = np.zeros(8, np.float64)
            r = lib.chain_ul_bench(0, v, T, n, R, len(pdus), arr, ptr(tbb), ptr(g), 4, 273, ptr(secs), 0.0, ptr(lat))
            assert r >= 0, r
            med = float(np.median(secs))
            run = {"variant": ["reference CPU processors", "GPU slot batch, synchronous",
                               "GPU service: 4 uplink processors per sector, asynchronous, "
                               "sectors aggregated per slot"][v], "threads": T,
                   "slots_per_thread": n, "seconds_median": med, "seconds": secs.tolist(),
                   "throughput_mbps_median": T * n * sum(tbs) / med / 1e6,
                   "slots_per_s": T * n / med,
                   # free-running: submission -> notification, queueing included (the paced section is the latency)
                   "latency_us_free_running": dict(zip(("p50", "p90", "p99", "max", "mean"), lat[:5]))}
            if pace_us > 0:
                # Real time: every sector submits a slot every pace_us (aligned, a radio's slot clock); the latency of
                # each PUSCH result from its slot's submission (handle_rx_symbol of the last symbol).
                lat = np.zeros(8, np.float64)
                r = lib.chain_ul_bench(0, v, T, n, 1, len(pdus), arr, ptr(tbb), ptr(g), 4, 273, ptr(secs), pace_us,
                                       ptr(lat))
                assert r >= 0, r
                run["paced"] = {"slot_period_us": pace_us, "seconds": float(secs[0]),
                                "kept_pace": bool(lat[7] < 5 * pace_us),
                                "max_submission_lag_us": float(lat[7]),
                                "latency_us": dict(zip(("p50", "p90", "p99", "max", "mean"), lat[:5])),
                                "over_5_slot_budget": float(lat[5]), "samples": int(lat[6])}
            case["runs"].append(run)
        out["ul"].append(case)
        print(json.dumps(case), file=sys.stderr, flush=True)

    def dl(name, pdus, tbs, weights):
        arr = (H.ChainParams * len(pdus))(*pdus)
        tbb = np.array(tbs, np.int32) // 8
        data = rng.integers(0, 256, int(tbb.sum())).astype(np.uint8)
        w = np.ascontiguousarray(np.concatenate([x.ravel() for x in weights]), np.complex64).view(np.float32)
        case = {"profile": name, "nof_pdus_per_slot": len(pdus), "tb_bits_per_slot": int(sum(tbs)), "runs": []}
        for v in (0, 1):
            n = slots
            secs = np.zeros(R, np.float64)
            r = lib.chain_dl_bench(0, v, T, n, R, len(pdus), arr, ptr(w), ptr(data), ptr(tbb), 4, 273, ptr(secs))
            assert r >= 0, r
            med = float(np.median(secs))
            case["runs"].append({"variant": ["reference CPU processors", "GPU slot batch"][v], "threads": T,
                                 "slots_per_thread": n, "seconds_median": med,
                                 "throughput_mbps_median": T * n * sum(tbs) / med / 1e6,
                                 "slots_per_s": T * n / med})
        out["dl"].append(case)
        print(json.dumps(case), file=sys.stderr, flush=True)

    # UL: the reference benchmark's PDU (273 PRB, 256QAM, 1 layer, random-noise grid) as one PDU per slot; 16 UEs.
    tbs = sch.tbs_calculate(273, 14, 6 * 2 * 2, 0, 8, 948.0, 1)
    p = H.params(slot=0, rnti=1, n_id=0, scrambling_id=0, nof_rb=273, rb_start=0, bwp_size=273, qm=8,
                 target_code_rate=948.0, nof_layers=1, nof_ports=4, base_graph=sch.base_graph(tbs, 948 / 1024),
                 tbs_lbrm_bytes=159749, max_iterations=2)
    if "ul" not in directions:
        ul = lambda *a: None  # noqa: E731
    if "dl" not in directions:
        dl = lambda *a: None  # noqa: E731
    ul("scs30_100MHz_256qam_rv0_4port_1layer, one PDU per slot", [p], [tbs])
    pdus, tb_list = [], []
    for i in range(16):
        u = sch.UeGrant(17, 1, 8, 948.0, nof_dmrs_symbols=2)
        seg = u.segmentation()
        pdus.append(H.params(rnti=0x4601 + i, harq_id=i, nof_rb=17, rb_start=17 * i, qm=8, target_code_rate=948.0,
                             nof_ports=4, base_graph=seg.base_graph, max_iterations=2))
        tb_list.append(seg.tbs)
    ul("16 UEs x 17 PRB, 256QAM, 1 layer (the slot processors' PUSCH PDU capacity)", pdus, tb_list)

    # DL: 270 PRB 4 layers on 4 ports as one PDU per slot; 16 UEs with 4 layers.
    tbs = sch.tbs_calculate(270, 12, 6 * 3 * 2, 0, 8, 948.0, 4)
    p = H.params(slot=0, rnti=1, n_id=0, scrambling_id=0, nof_rb=270, rb_start=0, bwp_size=273, qm=8,
                 target_code_rate=948.0, nof_layers=4, nof_ports=4, start_symbol=2, nof_symbols=12,
                 dmrs_mask=(1 << 2) | (1 << 7) | (1 << 11), base_graph=sch.base_graph(tbs, 948 / 1024),
                 tbs_lbrm_bytes=159749)
    q, _ = np.linalg.qr(rng.normal(size=(4, 4)) + 1j * rng.normal(size=(4, 4)))
    dl("4port_4layer_scs30_100MHz_256qam, one PDU per slot", [p], [tbs], [q.astype(np.complex64)])
    pdus, tb_list, ws = [], [], []
    for i in range(16):
        u = sch.UeGrant(17, 4, 8, 948.0, nof_symb_sh=12, nof_dmrs_symbols=2)
        seg = u.segmentation()
        pdus.append(H.params(rnti=0x4601 + i, nof_rb=17, rb_start=17 * i, qm=8, target_code_rate=948.0, nof_layers=4,
                             nof_ports=4, start_symbol=2, nof_symbols=12, dmrs_mask=(1 << 2) | (1 << 11),
                             base_graph=seg.base_graph))
        tb_list.append(seg.tbs)
        ws.append(np.eye(4, dtype=np.complex64))
    dl("16 UEs x 17 PRB, 256QAM, 4 layers (the slot processors' PDSCH UE PDU capacity)", pdus, tb_list, ws)
    return out


def main():
    import ctypes
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=host_cores())
    ap.add_argument("--batch", type=int, default=20)
    ap.add_argument("--repetitions", type=int, default=5)
    ap.add_argument("--slots", type=int, default=20, help="slot-processor section: slots per thread and repetition")
    ap.add_argument("--only-slots", action="store_true", help="run only the slot-processor section")
    ap.add_argument("--directions", default="ul,dl", help="slot-processor section: ul, dl or ul,dl")
    ap.add_argument("--pace-us", type=float, default=0.0,
                    help="slot-processor section, UL: also run every variant paced at one slot per this many us per "
                         "sector (500 = real time at 30 kHz) and report the PUSCH result latency")
    args = ap.parse_args()
    if args.only_slots:
        print(json.dumps({"threads": args.threads, "slot_processors": slot_cases(ctypes.CDLL(H.CHAIN_SO),
                                                                                args.threads, args.slots,
                                                                                args.repetitions,
                                                                                args.directions.split(","),
                                                                                args.pace_us)}))
        return
    lib = ctypes.CDLL(H.CHAIN_SO)
    PP = ctypes.POINTER(H.ChainParams)
    lib.chain_pusch_bench.restype = ctypes.c_int
    lib.chain_pusch_bench.argtypes = [ctypes.c_int, ctypes.c_int, PP, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint,
                                      ctypes.c_uint, ctypes.c_void_p]
    lib.chain_pdsch_bench.restype = ctypes.c_int
    lib.chain_pdsch_bench.argtypes = [ctypes.c_int, ctypes.c_int, PP, ctypes.c_void_p, ctypes.c_uint, ctypes.c_uint,
                                      ctypes.c_uint, ctypes.c_uint, ctypes.c_void_p]
    T, B, R = args.threads, args.batch, args.repetitions
    out = {"threads": T, "note": "reference processors (pusch_processor_impl / pdsch_processor_impl) on CPU components "
                                 "(mode 0) vs GPU bindings (PUSCH mode 2: GPU estimator + demodulator + "
                                 "pusch_decoder_hw_impl over the GPU accelerator; PDSCH mode 1: HW encoder + GPU "
                                 "modulator + GPU DM-RS); pusch_processor_benchmark.cpp / pdsch_processor_benchmark.cpp "
                                 "profiles, throughput_total = TB bits of all PDUs / wall time", "pusch": [], "pdsch": []}
    # PUSCH: scs30_100MHz_256qam_rv0_4port_nlayer (273 PRB, 256QAM R 948/1024, 4 rx ports, DM-RS 2 + 11, 2 CDM
    # groups, filter / interpolate / CFO estimator, 2 LDPC iterations, random-noise grid).
    for layers in (1, 2, 4):
        tbs = sch.tbs_calculate(273, 14, 6 * 2 * 2, 0, 8, 948.0, layers)
        p = H.params(slot=0, rnti=1, n_id=0, scrambling_id=0, nof_rb=273, rb_start=0, bwp_size=273, qm=8,
                     target_code_rate=948.0, nof_layers=layers, nof_ports=4, base_graph=sch.base_graph(tbs, 948 / 1024),
                     tbs_lbrm_bytes=159749)  # sch_constants.h:44 tbs_lbrm_default
        case = {"profile": "scs30_100MHz_256qam_rv0_4port_nlayer", "nof_prb": 273, "layers": layers, "tbs": tbs,
                "peak_mbps_per_cell": tbs / 500.0}
        modes = (0, 2) if layers == 1 else (2,)  # the reference's estimator estimates one layer
        case["runs"] = [run(lib, lib.chain_pusch_bench, m, p, tbs, T, B if m else max(2, B // 4), R) for m in modes]
        out["pusch"].append(case)
        print(json.dumps(case), file=sys.stderr, flush=True)
    # PDSCH: 4port_4layer_scs30_100MHz_256qam (270 PRB, 4 layers on 4 ports, symbols 2..13, DM-RS 2 + 7 + 11) and
    # scs30_100MHz_256qam_max (1 port, 1 layer).
    rng = np.random.default_rng(0)
    for name, layers in (("4port_4layer_scs30_100MHz_256qam", 4), ("scs30_100MHz_256qam_max", 1)):
        tbs = sch.tbs_calculate(270, 12, 6 * 3 * 2, 0, 8, 948.0, layers)
        p = H.params(slot=0, rnti=1, n_id=0, scrambling_id=0, nof_rb=270, rb_start=0, bwp_size=270, qm=8,
                     target_code_rate=948.0, nof_layers=layers, nof_ports=layers, start_symbol=2, nof_symbols=12,
                     dmrs_mask=(1 << 2) | (1 << 7) | (1 << 11), base_graph=sch.base_graph(tbs, 948 / 1024),
                     tbs_lbrm_bytes=159749)
        q, _ = np.linalg.qr(rng.normal(size=(layers, layers)) + 1j * rng.normal(size=(layers, layers)))
        case = {"profile": name, "nof_prb": 270, "layers": layers, "tbs": tbs, "peak_mbps_per_cell": tbs / 500.0}
        case["runs"] = [run(lib, lib.chain_pdsch_bench, m, p, tbs, T, B if m else max(2, B // 4), R, weights=q)
                        for m in (0, 1)]
        out["pdsch"].append(case)
        print(json.dumps(case), file=sys.stderr, flush=True)
    out["slot_processors"] = slot_cases(lib, T, args.slots, R)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
