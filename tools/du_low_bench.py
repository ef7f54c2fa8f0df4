#!/usr/bin/env python3
"""du_low on one GPU at the radio's pace. Uplink: S sectors, each a thread delivering its 100 MHz 4-port samples one
OFDM symbol per symbol duration to its lower-PHY PUxCH processor (row b5: one GPU processor per sector, or the sector
group), whose grid is the grid of one of the sector's uplink processors (row b6: the GPU slot batches on one shared
PUSCH service) with that slot's PUSCH PDUs; the last symbol of a slot starts the uplink processor, as du_low's
rx-symbol handler does (oracle/ref/ref_chain.cpp chain_du_low_ul). The PUSCH profiles are the reference benchmark's
(one 273-PRB 256QAM PDU, 2 LDPC iterations, on random-noise samples) and the slot processors' 16-UE capacity.

Reported per S: the largest lag behind the symbol pace, the lag at the end, the fraction of symbols more than a slot
late, late PUxCH requests and the PUSCH results notified; real time = every sector ends less than a slot behind with
under 1 % of its symbols a slot late and every PDU notified. Downlink (chain_du_low_dl): per sector an upper-PHY thread
runs the downlink processor (GPU PDSCH slot batch, one 270-PRB 4-layer PDU) for slot s + 2 while the radio thread takes
slot s's 14 symbols from the PDxCH processor, the grid going from the upper-PHY gateway to handle_request; real time as
for the UL, with every slot's symbols carrying samples and no late request. TEST INFRASTRUCTURE (diagnostic); GPU box:
    python tools/du_low_bench.py [--sectors 1,2,4,6,8] [--slots 200]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "srsran-5g_amd")]

import chain_harness as H  # noqa: E402
import lower_harness as LH  # noqa: E402
from srsgpu import sch  # noqa: E402

P, PRB, DFT = 4, 273, 4096


def profiles():
    tbs = sch.tbs_calculate(273, 14, 6 * 2 * 2, 0, 8, 948.0, 1)
    one = H.params(slot=0, rnti=1, n_id=0, scrambling_id=0, nof_rb=273, rb_start=0, bwp_size=273, qm=8,
                   target_code_rate=948.0, nof_layers=1, nof_ports=4, base_graph=sch.base_graph(tbs, 948 / 1024),
                   tbs_lbrm_bytes=159749, max_iterations=2)
    yield "one 273-PRB 256QAM PDU per slot", [one], [tbs]
    pdus, tb_list = [], []
    for i in range(16):
        u = sch.UeGrant(17, 1, 8, 948.0, nof_dmrs_symbols=2)
        seg = u.segmentation()
        pdus.append(H.params(rnti=0x4601 + i, harq_id=i, nof_rb=17, rb_start=17 * i, qm=8, target_code_rate=948.0,
                             nof_ports=4, base_graph=seg.base_graph, max_iterations=2))
        tb_list.append(seg.tbs)
    yield "16 UEs x 17 PRB per slot", pdus, tb_list


def dl_profiles(rng):
    tbs = sch.tbs_calculate(270, 12, 6 * 3 * 2, 0, 8, 948.0, 4)
    p = H.params(slot=0, rnti=1, n_id=0, scrambling_id=0, nof_rb=270, rb_start=0, bwp_size=273, qm=8,
                 target_code_rate=948.0, nof_layers=4, nof_ports=4, start_symbol=2, nof_symbols=12,
                 dmrs_mask=(1 << 2) | (1 << 7) | (1 << 11), base_graph=sch.base_graph(tbs, 948 / 1024),
                 tbs_lbrm_bytes=159749)
    q, _ = np.linalg.qr(rng.normal(size=(4, 4)) + 1j * rng.normal(size=(4, 4)))
    yield "one 270-PRB 4-layer 256QAM PDSCH per slot", [p], [tbs], [q.astype(np.complex64)]


def run_dl(lib, args, out):
    f = lib.chain_du_low_dl
    f.restype = ctypes.c_int
    f.argtypes = ([ctypes.c_int, ctypes.c_uint, ctypes.c_uint, ctypes.c_int, ctypes.POINTER(H.ChainParams)] +
                  [ctypes.c_void_p] * 3 + [ctypes.c_uint] * 3 + [ctypes.c_int] + [ctypes.c_void_p] * 3)
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    lib.chain_pdsch_transfer_counters.argtypes = [ctypes.c_void_p]

    def pdsch_twins():
        c = np.zeros(4, np.uint64)
        lib.chain_pdsch_transfer_counters(ptr(c))
        return int(c[3])

    rng = np.random.default_rng(6)
    for name, pdus, tbs, weights in dl_profiles(rng):
        arr = (H.ChainParams * len(pdus))(*pdus)
        tbb = np.array(tbs, np.int32) // 8
        data = rng.integers(0, 256, int(tbb.sum())).astype(np.uint8)
        w = np.ascontiguousarray(np.concatenate([x.ravel() for x in weights]), np.complex64).view(np.float32)
        for variant in args.variants.split(","):
            lower = "sector group" if variant == "group" else "one processor per sector"
            res = {"direction": "dl", "profile": name, "lower_phy": lower, "by_sectors": {}}
            for S in (int(v) for v in args.sectors.split(",")):
                lag = np.zeros((S, 4), np.float64)
                results = np.zeros((S, 2), np.int32)
                secs = np.zeros(1, np.float64)
                t0 = pdsch_twins()
                r = f(0, S, args.slots, len(pdus), arr, ptr(w), ptr(data), ptr(tbb), P, PRB, DFT,
                      1 if variant == "group" else 0, ptr(lag), ptr(results), ptr(secs))
                assert r == 0, r
                twins = pdsch_twins() - t0
                # every slot's 14 symbols but the first two slots' (requested before the run) carried samples
                complete = bool((results[:, 0] >= 14 * (args.slots - 2)).all())
                rt = bool(lag[:, 1].max() < 0.5e-3 and lag[:, 2].max() < 0.01 and complete and lag[:, 3].sum() == 0)
                res["by_sectors"][S] = {"max_lag_us": 1e6 * lag[:, 0].max(), "final_lag_us": 1e6 * lag[:, 1].max(),
                                        "late_fraction": lag[:, 2].max(), "late_requests": int(lag[:, 3].sum()),
                                        "symbols_with_samples": int(results[:, 0].sum()),
                                        "dl_slots_processed": int(results[:, 1].sum()), "complete": complete,
                                        "seconds": float(secs[0]), "real_time": rt,
                                        "grids_from_hbm_twin": twins}
                print(json.dumps({name: {variant: {S: res["by_sectors"][S]}}}), file=sys.stderr, flush=True)
            rts = [S for S, v in res["by_sectors"].items() if v["real_time"]]
            res["sectors_at_real_time"] = max(rts) if rts else 0
            out["runs"].append(res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--direction", default="ul,dl")
    ap.add_argument("--sectors", default="1,2,4,6,8")
    ap.add_argument("--slots", type=int, default=200)
    ap.add_argument("--in-flight", default="4,13")
    ap.add_argument("--variants", default="group,alone")
    args = ap.parse_args()
    lib = ctypes.CDLL(H.CHAIN_SO)
    f = lib.chain_du_low_ul
    f.restype = ctypes.c_int
    f.argtypes = ([ctypes.c_int, ctypes.c_uint, ctypes.c_uint, ctypes.c_int, ctypes.POINTER(H.ChainParams),
                   ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_uint] * 3 + [ctypes.c_int, ctypes.c_uint] +
                  [ctypes.c_void_p] * 4)
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    lib.chain_multi_transfer_counters.argtypes = [ctypes.c_void_p]

    def twin_grids():
        c = np.zeros(4, np.uint64)
        lib.chain_multi_transfer_counters(ptr(c))
        return int(c[3])
    n = sum(P * LH.symbol_size(1, DFT, False, s, l) for s in (0, 1) for l in range(14))
    rng = np.random.default_rng(5)
    samples = ((rng.normal(size=n) + 1j * rng.normal(size=n)) * 0.05).astype(np.complex64)
    out = {"config": {"sectors": "100 MHz 30 kHz 4T4R", "slots": args.slots}, "runs": []}
    if "dl" in args.direction:
        run_dl(lib, args, out)
    for name, pdus, tbs in (profiles() if "ul" in args.direction else ()):
        arr = (H.ChainParams * len(pdus))(*pdus)
        tbb = np.array(tbs, np.int32) // 8
        for variant in args.variants.split(","):
            for inflight in (int(v) for v in args.in_flight.split(",")):
                lower = "sector group" if variant == "group" else "one processor per sector"
                res = {"direction": "ul", "profile": name, "lower_phy": lower, "symbols_in_flight": inflight,
                       "by_sectors": {}}
                for S in (int(v) for v in args.sectors.split(",")):
                    lag = np.zeros((S, 4), np.float64)
                    results = np.zeros((S, 2), np.int32)
                    secs = np.zeros(1, np.float64)
                    lat = np.zeros(8, np.float64)
                    t0 = twin_grids()
                    r = f(0, S, args.slots, len(pdus), arr, ptr(tbb), ptr(samples), P, PRB, DFT,
                          1 if variant == "group" else 0, inflight, ptr(lag), ptr(results), ptr(secs), ptr(lat))
                    assert r == 0, r
                    twins = twin_grids() - t0
                    notified = bool((results[:, 0] == args.slots * len(pdus)).all())
                    rt = bool(lag[:, 1].max() < 0.5e-3 and lag[:, 2].max() < 0.01 and notified)
                    res["by_sectors"][S] = {"max_lag_us": 1e6 * lag[:, 0].max(), "final_lag_us": 1e6 * lag[:, 1].max(),
                                            "late_fraction": lag[:, 2].max(), "late_requests": int(lag[:, 3].sum()),
                                            "pusch_results": int(results[:, 0].sum()), "all_notified": notified,
                                            "seconds": float(secs[0]), "real_time": rt,
                                            # PUSCH result latency: end of the slot on the radio clock -> notification
                                            "latency_us": dict(zip(("p50", "p90", "p99", "max", "mean"), lat[:5])),
                                            "over_5_slot_budget": float(lat[5]),
                                            # slots whose rx grid the PUSCH launch found in HBM (written there by
                                            # the sector group's demodulation): no PCIe read-back
                                            "grids_from_hbm_twin": twins}
                    print(json.dumps({name: {variant: {inflight: {S: res["by_sectors"][S]}}}}), file=sys.stderr,
                          flush=True)
                rts = [S for S, v in res["by_sectors"].items() if v["real_time"]]
                res["sectors_at_real_time"] = max(rts) if rts else 0
                out["runs"].append(res)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
