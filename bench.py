#!/usr/bin/env python3
"""Benchmark: 100 MHz 4x4 PDSCH + PUSCH slot processing on MI355X (the whole upper-PHY data path plus OFDM).

BASELINE.json metric: "PDSCH+PUSCH slots/sec (100MHz 4x4) + LDPC info-bits/s at 1/2/4/8 GPU".
Workload ("n78 100 MHz 4x4, 273 PRB, LDPC BG1, batched 64 UEs"): one slot = 64 UEs sharing 273 PRBs (4-5 PRB each),
256QAM MCS 27 (table 2), DM-RS type 1 in symbols 2 and 11 (dmrs-AdditionalPosition pos1, two CDM groups without
data). A step processes `--slots-per-step` such slots per GPU, both directions, on two HIP streams (as a gNB runs
them concurrently):

  * DL (4 layers, 4 ports): PDSCH encoder (TB CRC, segmentation, CB CRC, LDPC, rate matching) -> PDSCH DM-RS ->
    PDSCH modulator (scrambling, 256QAM, layer mapping, precoding, RE mapping, bf16 grid) -> OFDM modulator
    (4096-point DFT, CP, phase compensation) of 4 ports: baseband samples.
  * UL (4 rx ports): OFDM demodulator -> DM-RS channel estimator (du_low defaults: filter smoothing, average time
    strategy, CFO estimation + compensation, time alignment) -> PUSCH demodulator (equalizer, soft demapping,
    descrambling) -> PUSCH decoder (rate dematching, LDPC min-sum, 6 iterations max with CRC early stop, SIMD
    arithmetic; TB CRC).

Profiles (--profile):
  * "ref" (default): every stage is one the open-source reference runs - single-layer PUSCH per UE (its estimator's
    limit, port_channel_estimator_average_impl.cpp:83) with ZF 1 x 4, so the GPU path and the cpu_baseline leg do the
    same, parity-pinned work (the bench checks the GPU's UL LLRs against the reference's on the same samples).
  * "mimo4": the extension - 4-layer PUSCH per UE (multi-layer estimation, 4 x 4 MMSE), beyond the reference.

Received samples: the UL transport blocks through a UE transmitter (the same GPU encoder / DM-RS / modulator), a
per-UE random unitary 4x4 channel, a per-UE CFO (+-300 Hz) and AWGN (--snr-db), OFDM-modulated; synthesised before
timing and resident in HBM. `--input-sets` independent copies of the whole per-step working set (TBs, samples, grids,
estimates, LLRs, HARQ buffers, decoded TBs, each set with its own plans and captured graph) are rotated step by step,
so the timed loop streams a working set larger than the 256 MB Infinity Cache. Operating points: the headline SNR,
plus `--extra-points` (a clean 35 dB link and the worst case: Gaussian noise, every codeblock runs all iterations,
like the reference's ldpc_decoder benchmark) timed the same way.

Workloads (--workload):
  * "multi_ue" (default, the headline): the 64-UE slot above, `--slots-per-step` slots per step in each direction.
  * "testmode": configs[4], the du_low test mode's traffic - one test UE owning all 273 PRB in every slot (max TBS:
    MCS 27, 4 DL layers), continuous slots of the du_high default TDD pattern DDDDDDSUUU (6 DL slots, a special slot
    with an 8-symbol PDSCH, 3 UL slots); a step is `--periods` TDD periods, value counts every slot of the pattern.
    Fresh DL payloads every step (drawn on the GPU inside the captured graph); the UL payloads differ per input set.

Weak scaling (--shard cells): every rank processes its own cells' slots; the decoded UL TBs + CRC flags of all ranks are
gathered to rank 0 (the FAPI rank) over RCCL once per step. Strong scaling (--shard ues): the 64 UEs of every slot are
split across the ranks (srsgpu.dist.shard_ues); rank 0 holds the cell's samples and runs its OFDM stages, the resource
grids are exchanged by subcarrier band (srsgpu.dist.GridExchange), each rank runs the upper PHY of its UEs, and the TBs
are gathered the same way. One JSON line from rank 0.
"""
import argparse
import ctypes
import json
import os
import sys
import threading
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
DMRS_MASK = slotlib.DMRS_POS1
CFO_HZ_MAX = 300.0

PROFILES = {
    "ref": dict(ul_layers=1, equalizer=srsgpu.EQ_ZF,
                ul_desc="single-layer PUSCH per UE, ZF 1x4 (the reference's estimator / equalizer scope)"),
    "mimo4": dict(ul_layers=4, equalizer=srsgpu.EQ_MMSE,
                  ul_desc="4-layer PUSCH per UE, multi-layer estimation + 4x4 MMSE (extension beyond the reference)"),
}


def host_cores():
    """Host cores this process may use: the affinity set, capped by OMP_NUM_THREADS (16 per GPU on the GPU box,
    where the affinity set shows the whole machine)."""
    n = len(os.sched_getaffinity(0))
    cap = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(cap))) if cap and cap.isdigit() else n


def cpu_baseline(dl_ues, dl_segs, ul_ues, ul_segs, tb_host, cw_host, samples_host, iterations, budget_s, cores,
                 tdd=None, ul_slot_index=0):
    """The srsRAN reference built from its own sources (oracle/_ref) on `cores` host threads, each running whole slots
    end to end with its own reference objects (slot-level parallelism: the best throughput the CPU path reaches on this
    workload): PDSCH encoding of the 64 DL TBs (pdsch_encoder_impl: segmenter + AVX2 LDPC encoder + rate matcher),
    PDSCH DM-RS + modulation of the 64 UEs into one grid and OFDM modulation of 4 ports (generic DFT), OFDM
    demodulation of 4 ports, per-UE DM-RS channel estimation (filter, average, CFO compensation) + PUSCH demodulation
    (single-layer ZF 1 x 4) of the same samples the GPU receives, and the PUSCH codeblock tasks (rate dematcher +
    LDPC decoder with CRC early stop, the implementations "auto" picks here) on the reference's own LLRs.
    `tdd` = (DL slots, UL slots) per TDD period (testmode): every thread still runs one DL and one UL slot per
    iteration; the period rate follows from the measured per-slot DL / UL shares (the special slot costed as a full DL
    slot, which favours the GPU's side of the ratio slightly less than the real 8-symbol PDSCH would).
    `ul_slot_index`: the frame slot number of the UL samples (DM-RS c_init, OFDM phase compensation).
    Returns (baseline dict, reference UL LLRs of slot 0, the reference decoder's iterations per codeblock of slot 0 on
    those LLRs, -1 where the CRC fails)."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libsrsref.so")
    if not os.path.exists(ref_so):
        return None, None, None
    lib = ctypes.CDLL(ref_so)
    P = ctypes.c_void_p
    for f in ("ref_pdsch_encode_slot_timed", "ref_pusch_decode_cbs_timed", "ref_dl_slot_timed", "ref_ul_slot_timed_at"):
        getattr(lib, f).restype = ctypes.c_longlong
    avx512 = bool(lib.ref_cpu_has_avx512())
    vbmi = bool(lib.ref_cpu_has_avx512vbmi())
    n = len(dl_ues)
    bg = np.array([s.base_graph for s in dl_segs], np.int32)
    qm = np.array([u.qm for u in dl_ues], np.int32)
    ly = np.array([u.nof_layers for u in dl_ues], np.int32)
    ns = np.array([u.nof_ch_symbols for u in dl_ues], np.uint32)
    tbb = np.array([s.tbs // 8 for s in dl_segs], np.uint32)
    nrb = np.array([u.n_prb for u in dl_ues], np.int32)
    rb0 = np.concatenate([[0], np.cumsum(nrb)[:-1]]).astype(np.int32)
    cw_off = np.array(cw_host[1], np.int32)
    ul_nrb = np.array([u.n_prb for u in ul_ues], np.int32)
    ul_rb0 = np.concatenate([[0], np.cumsum(ul_nrb)[:-1]]).astype(np.int32)
    params = []
    llr_off = 0
    for s in ul_segs:
        crc = 1 if s.nof_segments > 1 else (0 if s.tbs > 3824 else 3)
        for cb in s.codeblocks:
            params.append([s.base_graph, s.lifting_size, ul_ues[0].qm, cb.rm_length, cb.nof_filler_bits, crc,
                           cb.nof_crc_bits, llr_off + cb.cw_offset])
        llr_off += s.cw_length
    params = np.array(params, np.int32)
    nllr = llr_off

    def run_slot(st):
        cw = st["cw"]
        o1, o2 = ctypes.c_longlong(), ctypes.c_longlong()
        t = np.zeros(7)
        t[0] = lib.ref_pdsch_encode_slot_timed(1, n, bg.ctypes.data_as(P), qm.ctypes.data_as(P),
                                               ly.ctypes.data_as(P), ns.ctypes.data_as(P), tbb.ctypes.data_as(P),
                                               tb_host.ctypes.data_as(P), cw.ctypes.data_as(P))
        t[1] = lib.ref_dl_slot_timed(n, rb0.ctypes.data_as(P), nrb.ctypes.data_as(P), int(qm[0]), int(ly[0]),
                                     ctypes.c_uint(DMRS_MASK), cw_host[0].ctypes.data_as(P), cw_off.ctypes.data_as(P),
                                     ctypes.byref(o1))
        t[2] = o1.value
        t[3] = lib.ref_ul_slot_timed_at(len(ul_ues), ul_rb0.ctypes.data_as(P), ul_nrb.ctypes.data_as(P),
                                        int(ul_ues[0].qm), ctypes.c_uint(DMRS_MASK), 1, int(ul_slot_index),
                                        samples_host.ctypes.data_as(P), st["llr"].ctypes.data_as(P), ctypes.byref(o1),
                                        ctypes.byref(o2))
        t[4], t[5] = o1.value, o2.value
        t[6] = lib.ref_pusch_decode_cbs_timed(2 if vbmi else 1, 2 if avx512 else 1, len(params),
                                              params.ctypes.data_as(P), st["llr"].ctypes.data_as(P), iterations,
                                              st["iters"].ctypes.data_as(P))
        return t

    states = [{"cw": np.zeros(sum(s.cw_length for s in dl_segs), np.uint8), "llr": np.zeros(nllr, np.int8),
               "iters": np.zeros(len(params), np.int32), "slots": 0, "t": np.zeros(7), "it": []}
              for _ in range(cores)]
    start = threading.Barrier(cores + 1)
    stop = threading.Event()

    def worker(st):
        run_slot(st)  # untimed: first-call setup of the thread's reference objects (DFT plans, tables)
        start.wait()
        while not stop.is_set() or st["slots"] == 0:
            st["t"] += run_slot(st)
            st["slots"] += 1
            st["it"].append(np.where(st["iters"] > 0, st["iters"], iterations).mean())

    threads = [threading.Thread(target=worker, args=(st,)) for st in states]
    for th in threads:
        th.start()
    start.wait()
    t0 = time.perf_counter()
    time.sleep(budget_s)
    stop.set()
    for th in threads:
        th.join()
    wall = time.perf_counter() - t0
    slots = sum(st["slots"] for st in states)
    tt = sum(st["t"] for st in states) / slots * 1e-6  # ms per slot per thread, per stage
    it = float(np.mean([x for st in states for x in st["it"]]))
    value = slots / wall
    if tdd is not None:
        t_dl, t_ul = tt[0] + tt[1], tt[3] + tt[6]
        value = sum(tdd) / ((tdd[0] * t_dl + tdd[1] * t_ul) / (t_dl + t_ul) / value)
    base = {"value": value, "unit": "slots/s", "cores": cores, "kind": "reference",
            "sample": (f"TDD rate from {tdd[0]} DL + {tdd[1]} UL slots per period; " if tdd else "") +
                      f"{slots} DL+UL slot pairs in {wall:.1f} s on {cores} host threads, each running whole slots "
                      f"({len(dl_ues)} UEs) "
                      f"through the srsRAN reference with its own objects; per slot and thread: PDSCH encode "
                      f"{tt[0]:.2f} ms (avx2 encoder), PDSCH DM-RS + modulation {tt[1] - tt[2]:.2f} ms + OFDM "
                      f"modulation {tt[2]:.2f} ms (generic DFT), OFDM demodulation {tt[4]:.2f} ms + channel "
                      f"estimation {tt[5]:.2f} ms (filter, average, CFO compensation) + PUSCH demodulation "
                      f"{tt[3] - tt[4] - tt[5]:.2f} ms (single-layer ZF 1x4), PUSCH codeblock tasks {tt[6]:.2f} ms "
                      f"({'avx512' if vbmi else 'avx2'} dematcher, {'avx512' if avx512 else 'avx2'} decoder, "
                      f"{iterations} iterations max, early stop, avg {it:.2f} iterations)"}
    return base, states[0]["llr"].copy(), states[0]["iters"].copy()


def reference_build_spread(ul_ues, samples_host, ul_slot_index, ref_llr):
    """The reference's own reproducibility on the UL slot of the LLR parity check: the same samples through the
    reference built at -march=x86-64-v4 (AVX-512; oracle/build_ref.sh SRSREF_MARCH) against its AVX2 + FMA build (the
    one `cpu_baseline` runs). Its srsvec reductions change order with the SIMD width, so its LLRs move by a few steps
    between builds (tests/test_reference_isa_variance.py). None when that build or an AVX-512 host is absent."""
    so = os.path.join(ROOT, "oracle", "_ref", "libsrsref_x86-64-v4.so")
    if ref_llr is None or not os.path.exists(so):
        return None
    lib = ctypes.CDLL(so)
    if not lib.ref_cpu_has_avx512():
        return None
    P = ctypes.c_void_p
    lib.ref_ul_slot_timed_at.restype = ctypes.c_longlong
    ul_nrb = np.array([u.n_prb for u in ul_ues], np.int32)
    ul_rb0 = np.concatenate([[0], np.cumsum(ul_nrb)[:-1]]).astype(np.int32)
    llr = np.zeros_like(ref_llr)
    o1, o2 = ctypes.c_longlong(), ctypes.c_longlong()
    lib.ref_ul_slot_timed_at(len(ul_ues), ul_rb0.ctypes.data_as(P), ul_nrb.ctypes.data_as(P), int(ul_ues[0].qm),
                             ctypes.c_uint(DMRS_MASK), 1, int(ul_slot_index), samples_host.ctypes.data_as(P),
                             llr.ctypes.data_as(P), ctypes.byref(o1), ctypes.byref(o2))
    d = np.abs(llr.astype(np.int16) - ref_llr.astype(np.int16))
    return {"builds": "reference -march=x86-64-v4 vs its -mavx2 -mfma build", "equal": float(np.mean(d == 0)),
            "within_one_step": float(np.mean(d <= 1)), "max_diff": int(d.max()), "over_one_step": int(np.sum(d > 1))}


class InputSet:
    """One independent copy of a step's working set: DL / UL pipelines (plans + buffers), DL TBs, UL samples and the
    UL TBs the UEs sent. Sets are rotated step by step. `dl_cells`: the DL slot groups of a step (one, or a TDD
    period's full and special slots), run as one DownlinkGroup."""

    def __init__(self, ctx, dl_cells, ul_cell, prof, iterations, gen, dev, fresh_tbs=False):
        self.dls = [slotlib.DownlinkPipeline(ctx, c) for c in dl_cells]
        self.dl = self.dls[0]
        self.ul = slotlib.UplinkPipeline(ctx, ul_cell, iterations=iterations, equalizer=prof["equalizer"],
                                         compensate_cfo=True)
        # Padded to 8 bytes: fresh payloads are drawn 8 bytes at a time (the plans read tb_total bytes).
        self.dl_tbs_all = [torch.randint(0, 256, ((d.tb_total + 7) // 8 * 8,), generator=gen, device=dev,
                                         dtype=torch.uint8) for d in self.dls]
        self.dl_tbs = self.dl_tbs_all[0]
        self.dl_group = slotlib.DownlinkGroup(self.dls, self.dl_tbs_all, fresh_tbs=fresh_tbs)
        self.ul_tbs_tx = torch.randint(0, 256, (sum(self.ul.tb_bytes),), generator=gen, device=dev,
                                       dtype=torch.uint8)
        self.samples = torch.zeros(2 * self.ul.ofdm.nof_samples, dtype=torch.float32, device=dev)
        self.graph = None
        self.graph_back = None  # UE-sharded cell: the part after the grid exchange
        self.graph_ul = None    # --leg-graphs: the UL leg's own graph (self.graph then holds the DL leg)
        self.tb_gather = None   # srsgpu.dist.TbGather of this set (ranks > 1)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # A minimum: the headline loop is extended until it has run for --min-time seconds (the actual count is reported).
    ap.add_argument("--steps", type=int, default=4000)
    ap.add_argument("--min-time", type=float, default=1.0, help="seconds the headline timed loop runs at least")
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--profile", choices=sorted(PROFILES), default="ref")
    ap.add_argument("--workload", choices=["multi_ue", "testmode"], default="multi_ue")
    # testmode: 4 TDD periods per step (40 slots, 0.18 ms); MI355X sweep: 2 periods 142.7k (5 sets) / 159.2k (3 sets),
    # 4 periods 227.9k slots/s (profiles/r2_step_shape_sweep.txt).
    ap.add_argument("--periods", type=int, default=4, help="testmode: TDD periods (10 slots each) per step")
    # A step is a batch of 32 slots (at ~60 cells per GPU, one slot of 32 cells of a slot period, 0.27 ms < 0.5 ms);
    # 5 input sets in flight: sweep on MI355X (profiles/r2_step_shape_sweep.txt): 16 / 4 88.0k, 16 / 2 106.2k,
    # 32 / 2 117.9k, 32 / 4 103.8k, 32 / 5 117.9k, 64 / 3 120.5k slots/s (set counts that are multiples of the 4
    # hardware queues serialise the sets' graph branches).
    ap.add_argument("--slots-per-step", type=int, default=32)
    ap.add_argument("--input-sets", type=int, default=13, help="independent working sets rotated step by step")
    ap.add_argument("--iterations", type=int, default=6)
    ap.add_argument("--snr-db", type=float, default=26.0)
    ap.add_argument("--worst-case", action="store_true", help="headline on Gaussian-noise input (all iterations)")
    ap.add_argument("--extra-points", action=argparse.BooleanOptionalAction, default=True,
                    help="also time the 35 dB and worst-case operating points (--point-steps steps each)")
    ap.add_argument("--point-steps", type=int, default=1000)
    ap.add_argument("--extra-workloads", action=argparse.BooleanOptionalAction, default=True,
                    help="after the headline, also measure the 4-layer mimo4 profile and the test mode (configs[4]) "
                         "in the same run, each with its own roofline (field 'workloads')")
    ap.add_argument("--shard", choices=["cells", "ues"], default="cells")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--serial-legs", action="store_true",
                    help="run the DL and UL legs on one stream (clean per-stage times; slower overall)")
    ap.add_argument("--pipeline", action=argparse.BooleanOptionalAction, default=True,
                    help="replay each input set on its own stream (up to --input-sets steps in flight)")
    ap.add_argument("--graph", action=argparse.BooleanOptionalAction, default=True,
                    help="replay each set's DL+UL pipeline as one captured HIP graph (default) or launch eagerly")
    # Two graphs per set, each leg on its own stream, with 9 sets: 134.3k slots/s vs 130.0k for one graph per set
    # with 5 sets (profiles/r3_leg_graphs_sweep.json: one graph per set with 7 sets drops to 123k; 7-14 sets with leg
    # graphs give 132.9k-135.0k).
    ap.add_argument("--dl-priority", type=int, default=int(os.environ.get("SRSGPU_BENCH_DL_PRIORITY", "0")),
                    help="1: replay each set's step (the DL leg with --leg-graphs) on high-priority streams")
    ap.add_argument("--ul-priority", type=int, default=int(os.environ.get("SRSGPU_BENCH_UL_PRIORITY", "0")),
                    help="1: replay the UL legs on high-priority streams (with --leg-graphs)")
    ap.add_argument("--leg-graphs", action=argparse.BooleanOptionalAction, default=True,
                    help="capture the DL and UL legs of a step as two graphs replayed on two streams per input set")
    ap.add_argument("--graph-collectives", action=argparse.BooleanOptionalAction, default=True,
                    help="capture the RCCL exchanges (TB gather; grid exchange with --shard ues) inside the step's "
                         "graphs (default) instead of issuing them between graph launches")
    ap.add_argument("--tb-gather", choices=["auto", "always", "never"], default="auto",
                    help="the per-step TB gather to the FAPI rank: with more than one rank (auto), also at world size "
                         "1 under torchrun (always: exercises RCCL graph capture on one GPU), or never")
    return ap.parse_args(argv)


def _load_keyed(path, wl_key):
    """A committed profile summary (profiles/*.json) for workload wl_key: either a single-workload file
    ({"workload": key, ...}) or {"by_workload": {key: {...}}}."""
    if not os.path.exists(path):
        return None
    with open(path) as f:
        j = json.load(f)
    if j.get("workload") == wl_key:
        return j
    return j.get("by_workload", {}).get(wl_key)


def measure(args, env):
    """One workload / profile measured end to end: build the input sets, warm up, capture, the timed loop (extended to
    --min-time), roofline of the dominant kernel, operating points, and (rank 0, one GPU) the reference CPU leg with
    the UL LLR parity check. Returns the result dict (rank 0's is printed)."""
    prof = PROFILES[args.profile]
    ctx, dev, gen, world, rank = env["ctx"], env["dev"], env["gen"], env["world"], env["rank"]
    S = args.slots_per_step
    K = max(1, args.input_sets)

    dl_all = sch.slot_100mhz_4x4(nof_layers=4, nof_dmrs_symbols=2)
    ul_all = sch.slot_100mhz_4x4(nof_layers=prof["ul_layers"], nof_dmrs_symbols=2)
    testmode = args.workload == "testmode"
    if testmode and args.shard == "ues" and world > 1:
        raise SystemExit("--workload testmode has one UE per slot: --shard ues does not apply")
    if testmode:
        dl_cell, sp_cell, ul_cell = slotlib.tdd_testmode_cells(args.periods, 4, prof["ul_layers"])
        dl_cells = [dl_cell, sp_cell]
        dl_ues, ul_ues, dl_segs, ul_segs = dl_cell.ues, ul_cell.ues, dl_cell.segs, ul_cell.segs
    elif args.shard == "ues" and world > 1:
        from srsgpu import dist as sdist
        dl_ues, ul_ues = sdist.shard_ues(dl_all, world, rank), sdist.shard_ues(ul_all, world, rank)
        rb_first = sum(u.n_prb for u in dl_all[:sdist.shard_range(len(dl_all), world, rank).start])
    else:
        dl_ues, ul_ues, rb_first = dl_all, ul_all, 0
    if not testmode:
        dl_segs = [u.segmentation() for u in dl_ues]
        ul_segs = [u.segmentation() for u in ul_ues]
        dl_cell = slotlib.CellSlots(dl_ues, dl_segs, S, dmrs_mask=DMRS_MASK, rb_first=rb_first)
        ul_cell = slotlib.CellSlots(ul_ues, ul_segs, S, dmrs_mask=DMRS_MASK, rb_first=rb_first)
        dl_cells = [dl_cell]
    # Slots a step processes (value's unit): a TDD period's slots in testmode, else the slots of each direction.
    slots_per_step = args.periods * slotlib.TDD_PERIOD if testmode else S
    S_ul = ul_cell.nof_slots
    S_dl = sum(c.nof_slots for c in dl_cells)
    sets = [InputSet(ctx, dl_cells, ul_cell, prof, args.iterations, gen, dev, fresh_tbs=testmode) for _ in range(K)]
    # UE-sharded cell (strong scaling): the cell's samples enter and leave on rank 0, which runs the OFDM stages of the
    # whole cell; the resource grids are exchanged by subcarrier band (srsgpu.dist.GridExchange: UL scatter after the
    # OFDM demodulation, DL gather before the OFDM modulation). Rank 0 synthesises the whole cell's UL from the TBs of
    # all UEs (drawn identically on every rank); each rank checks its own UEs' decoded TBs.
    shard_x = args.shard == "ues" and world > 1
    if shard_x:
        from srsgpu import dist as sdist
        full_ul_cell = slotlib.CellSlots(ul_all, [u.segmentation() for u in ul_all], S, dmrs_mask=DMRS_MASK)
        full_bytes = [s.tbs // 8 for s in full_ul_cell.segs]
        mine = sdist.shard_range(len(ul_all), world, rank)
        off0, n_r, tot = sum(full_bytes[:mine.start]), sum(full_bytes[mine.start:mine.stop]), sum(full_bytes)
        for k, st in enumerate(sets):
            g_all = torch.Generator(device=dev)
            g_all.manual_seed(777 + k)
            st.full_ul_tbs = torch.randint(0, 256, (S * tot,), generator=g_all, device=dev, dtype=torch.uint8)
            st.ul_tbs_tx = torch.cat([st.full_ul_tbs[s * tot + off0: s * tot + off0 + n_r] for s in range(S)])
        ranges = sdist.ue_subcarrier_ranges(ul_all, world)
        gx_ul = sdist.GridExchange(S * ul_cell.nof_ports * 14, ul_cell.nsc, ranges, dev, root=0)
        gx_dl = sdist.GridExchange(S * dl_cell.nof_ports * 14, dl_cell.nsc, ranges, dev, root=0)

    def fill_samples(snr_db, worst):
        for k, st in enumerate(sets):
            if shard_x and rank != 0:
                continue  # only the root rank receives the cell's samples
            if worst:
                st.samples.copy_(torch.randn(st.samples.numel(), generator=gen, device=dev) * 0.01)
            elif shard_x:
                st.samples.copy_(slotlib.synthesize_uplink(ctx, full_ul_cell, st.full_ul_tbs, snr_db=snr_db,
                                                           seed=99 + 1000 * k, cfo_hz_max=CFO_HZ_MAX))
            else:
                st.samples.copy_(slotlib.synthesize_uplink(ctx, ul_cell, st.ul_tbs_tx, snr_db=snr_db,
                                                           seed=99 + rank + 1000 * k, cfo_hz_max=CFO_HZ_MAX))
        torch.cuda.synchronize()

    fill_samples(args.snr_db, args.worst_case)
    dl_stream = torch.cuda.Stream(dev)
    ul_stream = dl_stream if args.serial_legs else torch.cuda.Stream(dev)
    # The decoded TBs + CRC flags of every rank go to the FAPI rank once per step (srsgpu.dist.TbGather). One gather
    # per input set: each set's step runs on its own streams, so sets must not share send / receive buffers.
    use_gather = dist.is_available() and dist.is_initialized() and (world > 1 or args.tb_gather == "always")
    if use_gather and args.tb_gather != "never":
        from srsgpu import dist as sdist
        for st in sets:
            st.tb_gather = sdist.TbGather(st.ul.d_tbs.numel(), st.ul.d_tb_ok.numel(), dev, root=0)
    tb_gather = sets[0].tb_gather

    def pipeline(st, ev_dl=None, ev_ul=None, part="all"):
        """DL and UL legs of one step of input set `st`, forked from and joined back into the current stream. A
        UE-sharded cell runs it as part "front" (DL upper PHY into the grids; UL OFDM demodulation on the root),
        the grid exchange (`exchange`) and part "back" (DL OFDM modulation on the root; UL upper PHY)."""
        cur = torch.cuda.current_stream(dev)
        dl_stream.wait_stream(cur)
        ul_stream.wait_stream(cur)
        root = rank == 0
        if part == "all":
            st.dl_group.execute(dl_stream, ev_dl)
            st.ul.execute(st.samples, ul_stream, ev_ul)
        elif part == "front":
            st.dl_group.execute(dl_stream, ev_dl, upper=True, back=False)
            st.ul.execute(st.samples, ul_stream, ev_ul, ofdm=root, upper=False)
        else:
            st.dl_group.execute(dl_stream, ev_dl, upper=False, ofdm=root)
            st.ul.execute(None, ul_stream, ev_ul, upper=True, front=False)
        cur.wait_stream(dl_stream)
        cur.wait_stream(ul_stream)

    def exchange(st):
        """UE-sharded cell: the DL grid bands to the root, the root's UL grid bands to their ranks (current stream)."""
        gx_dl.gather(st.dls[0].d_grid)
        gx_ul.scatter(st.ul.d_grid)

    def whole(st, ev_dl=None, ev_ul=None):
        if shard_x:
            pipeline(st, ev_dl, ev_ul, "front")
            exchange(st)
            pipeline(st, ev_dl, ev_ul, "back")
        else:
            pipeline(st, ev_dl, ev_ul)

    # Pipelining across steps: each input set replays on its own stream, so a step's UL decode can overlap the next
    # set's front end (different buffers; a set's consecutive steps stay ordered on its stream).
    set_streams = ([torch.cuda.Stream(dev, priority=-args.dl_priority) for _ in range(K)]
                   if args.pipeline else None)
    # --leg-graphs: the DL and UL legs of a set as two graphs replayed on two streams of their own.
    leg_graphs = args.leg_graphs and args.graph and not shard_x
    # --ul-priority: the UL legs' streams at a higher HIP stream priority (-1), so the decoder's workgroups are
    # dispatched ahead of the DL leg's when both wait for a CU.
    ul_set_streams = ([torch.cuda.Stream(dev, priority=-args.ul_priority) for _ in range(K)]
                      if leg_graphs and args.pipeline else None)

    def step(i):
        st = sets[i % K]
        cur = torch.cuda.current_stream(dev) if set_streams is None else set_streams[i % K]
        if st.graph_ul is not None:
            cur_ul = cur if ul_set_streams is None else ul_set_streams[i % K]
            with torch.cuda.stream(cur):
                st.graph.replay()
            with torch.cuda.stream(cur_ul):
                st.graph_ul.replay()
                if st.tb_gather is not None and not args.graph_collectives:
                    st.tb_gather.gather(st.ul.d_tbs, st.ul.d_tb_ok)
            return
        with torch.cuda.stream(cur):
            if st.graph is not None and st.graph_back is not None:
                st.graph.replay()     # front part
                exchange(st)          # RCCL grid exchange between the captured parts
                st.graph_back.replay()
            elif st.graph is not None:
                st.graph.replay()
            else:
                whole(st)
            if st.tb_gather is not None and not (st.graph is not None and args.graph_collectives):
                st.tb_gather.gather(st.ul.d_tbs, st.ul.d_tb_ok)

    # Every input set runs at least once before timing (its buffers, plans and code first touched), whatever --warmup.
    n_warm = max(args.warmup, K)
    for i in range(n_warm):
        step(i)
    torch.cuda.synchronize()
    skip = [s for s in os.environ.get("SRSGPU_BENCH_SKIP", "").split(",") if s]
    if skip:
        # Timing experiment only (stage sensitivity: how much of the overlapped step each stage costs): the named
        # stages' launches are dropped from the captured step; their outputs keep the warm-up's values (same inputs
        # every step). The line is marked and is not a valid measurement.
        for st in sets:
            plans = {"encode": [d.encoder for d in st.dls], "dmrs": [d.dmrs for d in st.dls],
                     "modulate": [d.modulator for d in st.dls], "ofdm_mod": [d.ofdm for d in st.dls],
                     "ofdm_demod": [st.ul.ofdm], "chest": [st.ul.chest], "demod": [st.ul.demod],
                     "decode": [st.ul.decoder]}
            for s in skip:
                for p in plans[s]:
                    p.execute = lambda *a, **k: None
    if args.graph:
        # One hipGraph per input set of the whole per-step pipeline (every plan is allocation-free and capture-safe):
        # the kernels, the codeword memset and the stream fork/join replay as one graph launch per step.
        # thread_local: the RCCL watchdog thread of a multi-GPU run keeps polling its events during the capture.
        for st in sets:
            st.graph = torch.cuda.CUDAGraph()
            if leg_graphs:
                with torch.cuda.graph(st.graph, capture_error_mode="thread_local"):
                    st.dl_group.execute(torch.cuda.current_stream(dev))
                st.graph_ul = torch.cuda.CUDAGraph()
                with torch.cuda.graph(st.graph_ul, capture_error_mode="thread_local"):
                    st.ul.execute(st.samples, torch.cuda.current_stream(dev))
                    if st.tb_gather is not None and args.graph_collectives:
                        # RCCL graph capture: the gather replays with the UL leg, on its stream.
                        st.tb_gather.gather(st.ul.d_tbs, st.ul.d_tb_ok)
            elif shard_x and not args.graph_collectives:
                # The collectives stay outside: the front and back parts are captured as two graphs.
                with torch.cuda.graph(st.graph, capture_error_mode="thread_local"):
                    pipeline(st, part="front")
                st.graph_back = torch.cuda.CUDAGraph()
                with torch.cuda.graph(st.graph_back, capture_error_mode="thread_local"):
                    pipeline(st, part="back")
            else:
                # --graph-collectives: the grid exchange and the TB gather are captured with the kernels (RCCL graph
                # capture); otherwise there are no collectives in the step's kernels.
                with torch.cuda.graph(st.graph, capture_error_mode="thread_local"):
                    whole(st)
                    if st.tb_gather is not None and args.graph_collectives:
                        st.tb_gather.gather(st.ul.d_tbs, st.ul.d_tb_ok)
        for i in range(n_warm):
            step(i)
        torch.cuda.synchronize()

    def timed(steps):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            step(i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def timed_min(steps, min_time):
        """timed(steps), re-run with proportionally more steps when it took less than min_time (the same count on
        every rank: the elapsed time is already the max over ranks). Returns (steps actually timed, seconds)."""
        e = timed(steps)
        if e < min_time:
            steps = int(np.ceil(steps * 1.1 * min_time / max(e, 1e-6)))
            e = timed(steps)
        return steps, e

    def ul_results(check_payload):
        """UL TB success and LDPC iterations of the last step of every set; decoded TBs with a passing CRC must
        equal what the UEs sent."""
        ok_all, it_all = [], []
        for st in sets:
            ok = st.ul.d_tb_ok.cpu().numpy().astype(bool)
            it = st.ul.d_iters.cpu().numpy()
            if check_payload:
                sent, got, off = st.ul_tbs_tx.cpu().numpy(), st.ul.d_tbs.cpu().numpy(), 0
                for i, nb in enumerate(st.ul.tb_bytes):
                    if ok[i]:
                        assert np.array_equal(got[off:off + nb], sent[off:off + nb]), f"TB {i} CRC ok, payload differs"
                    off += nb
            ok_all.append(ok)
            it_all.append(np.where(it > 0, it, args.iterations))
        return float(np.concatenate(ok_all).mean()), float(np.concatenate(it_all).mean())

    steps, elapsed = timed_min(args.steps, args.min_time)
    tb_success, avg_iters = ul_results(not args.worst_case)
    agg = world if args.shard == "cells" else 1  # ranks whose slots add up (weak scaling)
    step_rate = agg * steps / elapsed            # steps/s of the whole job
    value = slots_per_step * step_rate

    # Roofline kernel time: an eager pass over the sets with the decoder plans' own stage events (the decoding launch
    # on its stream), right after the timed loop.
    st0 = sets[0]
    for st in sets:
        st.ul.decoder.stage_times()
        st.ul.decoder.enable_timing(True, decode_only=True)
    n_dec = min(steps, 400)
    for i in range(n_dec):
        whole(sets[i % K])
    torch.cuda.synchronize()
    dec_ms_tot, dec_n = 0.0, 0
    for st in sets:
        ms, n = st.ul.decoder.stage_times()
        dec_ms_tot += ms[1]
        dec_n += n
        st.ul.decoder.enable_timing(False)
    assert dec_n == n_dec or "decode" in skip
    dec_ms = dec_ms_tot / dec_n if dec_n else float("nan")
    # Per-stage times: another untimed eager pass with events between the stages.
    n_stage = min(steps, 200)
    evs = [([torch.cuda.Event(enable_timing=True) for _ in range(4)],
            [torch.cuda.Event(enable_timing=True) for _ in range(5)]) for _ in range(n_stage)]
    for i in range(n_stage):
        whole(sets[i % K], *evs[i])
    torch.cuda.synchronize()
    stage = {k: 0.0 for k in DL_STAGES + UL_STAGES}
    for ed, eu in evs:
        for j, k in enumerate(DL_STAGES):
            stage[k] += ed[j].elapsed_time(ed[j + 1]) / n_stage
        for j, k in enumerate(UL_STAGES):
            stage[k] += eu[j].elapsed_time(eu[j + 1]) / n_stage

    # ---- Operating points: the same timed loop on other inputs (samples rewritten in place; graphs unchanged) ----
    points = [{"name": "headline", "snr_db": None if args.worst_case else args.snr_db, "value": value,
               "ms_per_step": elapsed * 1e3 / steps, "steps": steps,
               "pusch_tb_success_rate": tb_success, "ldpc_avg_iterations": avg_iters}]
    if args.extra_points:
        for name, snr, worst in (("clean_35dB", 35.0, False), ("worst_case_noise", None, True)):
            fill_samples(snr, worst)
            for i in range(max(args.warmup, K)):
                step(i)
            ps, e = timed_min(args.point_steps, args.min_time / 2)
            ok, it = ul_results(not worst)
            points.append({"name": name, "snr_db": snr, "value": slots_per_step * agg * ps / e,
                           "ms_per_step": e * 1e3 / ps, "steps": ps, "pusch_tb_success_rate": ok,
                           "ldpc_avg_iterations": it})
        fill_samples(args.snr_db, args.worst_case)

    # ---- Roofline of the dominant kernel (LDPC decoder) ----
    ul, dl = st0.ul, st0.dl
    info_bits_slot = sum(((22 if s.base_graph == 1 else 10) * s.lifting_size - s.nof_filler_bits) * s.nof_segments
                         for s in ul_segs)
    tbs_bits_ul_step = sum(s.tbs for s in ul_segs) * S_ul
    tbs_bits_dl_step = sum(sum(s.tbs for s in c.segs) * c.nof_slots for c in dl_cells)
    # Algorithmic bytes of one decoder launch: the LLRs each codeblock's decode() reads (the HARQ span up to the
    # dematcher's zero tail, as reported by the plan), K*Z/8 bytes of decoded bits written, 4 B result + 1 B CRC flag,
    # 40 B descriptor.
    dec_bytes = ul.decoder.decoder_input_llrs + sum(
        s.nof_segments * (((22 if s.base_graph == 1 else 10) * s.lifting_size + 7) // 8 + 45) for s in ul_segs) * S_ul
    achieved = dec_bytes / (dec_ms * 1e-3) / 1e9
    wl_key = (f"testmode/P{args.periods}/" if testmode else "") + \
        f"{args.profile}/S{S}/{'noise' if args.worst_case else f'{args.snr_db:g}dB'}"
    tj = _load_keyed(os.path.join(ROOT, "profiles", "ldpc_decode_traffic.json"), wl_key)
    traffic = tj.get("hbm_bytes_per_launch") if tj else None
    # VALU roofline of the same launch: wave-level VALU instructions per launch from the committed SQ counter pass
    # (rocprofv3 --pmc SQ_INSTS_VALU ..., tools/sq_summary.py; same workload) over the live kernel time.
    valu = None
    dec_kernel = "ldpc_decode_pk_kernel (plain or edge-split variant)"
    sqj = _load_keyed(os.path.join(ROOT, "profiles", "sq_valu.json"), wl_key)
    if sqj:
        sq_name, sq = next(((k, v) for k, v in sqj.get("kernels", {}).items() if k.startswith("ldpc_decode")),
                           (None, None))
        if sq_name:
            dec_kernel = sq_name.replace(" ", "")
        if sq:
            peak = 1024 * 2.4e9 / 2  # SIMDs x clock / 2 cycles per wave64 VALU instruction (MI355X_MICROARCH.md)
            # Measured ceiling of the decoder's instruction mix (profiles/r3_valu_rate_probe_*.log: independent
            # v_pk_* streams saturate at 2.2 G wave-instr/s per CU, VOP2 at 3.4; 80 / 20 % mix -> 2.35 G/s per CU).
            mix_peak = 256 * 2.35e9
            rate = sq["valu_instr"] / (dec_ms * 1e-3)
            valu = {"bound": "valu_issue", "achieved": rate, "peak": peak, "unit": "wave-instr/s",
                    "frac": rate / peak, "instr_per_launch": sq["valu_instr"],
                    "peak_measured_mix": mix_peak, "frac_of_measured_mix_peak": rate / mix_peak,
                    "source": "profiles/sq_valu.json (SQ_INSTS_VALU) / live kernel time; peak = 2 cycles per wave64 "
                              "instruction on SIMD-32; peak_measured_mix = the rate probe's ceiling for 80 % packed "
                              "16-bit (v_pk_*, ~3.9 cycles each) + 20 % 32-bit VALU"}

    # Algorithmic HBM bytes per step of the signal-chain stages (each byte read or written once; DESIGN.md "Kernels"):
    # bf16 grids are 4 B per RE, time samples 8 B (complex float), estimates 4 B per (layer, port, RE), LLRs 1 B.
    P, nsc, Lu = ul_cell.nof_ports, ul_cell.nsc, prof["ul_layers"]
    grid_b_dl, grid_b_ul = S_dl * P * 14 * nsc * 4, S_ul * P * 14 * nsc * 4
    spp = ul.ofdm.nof_samples // (S_ul * P)  # samples per slot and port (CPs included)
    nd = bin(DMRS_MASK).count("1")
    data_re = S_ul * sum(12 * u.n_prb * (14 - nd) for u in ul_ues)
    cw_b = sum(sum(s.cw_length for s in c.segs) * c.nof_slots for c in dl_cells) // 8
    ce_rows = 1 if ul.estimate_layout == srsgpu.CE_COMPACT else 14
    ce_b = S_ul * Lu * P * ce_rows * 12 * sum(u.n_prb for u in ul_ues) * 4
    stage_bytes = {
        "pdsch_dmrs_modulate": cw_b + grid_b_dl,
        "ofdm_modulate": grid_b_dl + S_dl * P * spp * 8,
        "ofdm_demodulate": S_ul * P * 14 * slotlib.DFT_SIZE * 8 + grid_b_ul,
        "pusch_channel_estimate": S_ul * P * nd * nsc * 4 + ce_b,
        "pusch_demodulate": data_re * (P * 4 + Lu * ul_ues[0].qm) + ce_b,
        # TB bytes read + codeword bytes written
        "pdsch_encode": sum(sum(s.tbs for s in c.segs) * c.nof_slots for c in dl_cells) // 8 + cw_b,
    }
    stage_gbps = {k: v / (stage[k] * 1e-3) / 1e9 for k, v in stage_bytes.items() if stage[k] > 0}
    set_bytes = sum(t.numel() * t.element_size() for t in
                    [*st0.dl_tbs_all, st0.samples, st0.ul_tbs_tx, ul.d_grid, ul.d_nv, ul.d_llrs, ul.d_harq, ul.d_crc,
                     ul.d_msgs, ul.d_iters, ul.d_tbs, ul.d_tb_ok]
                    + [t for d in st0.dls for t in (d.d_cw, d.d_grid, d.d_samples)]) \
        + S_ul * Lu * P * 14 * nsc * 4 // 14 * ce_rows
    if testmode:
        workload = (f"du_low test mode (configs[4]): n78 100 MHz 4x4, one test UE x 273 PRB per slot (max TBS), "
                    f"256QAM MCS27, TDD DDDDDDSUUU x {args.periods} per step (special slot: 8-symbol PDSCH, DM-RS "
                    f"2+7); DM-RS symbols 2+11; DL 4 layers, UL {prof['ul_desc']}; LDPC BG1; fresh DL payloads "
                    f"every step")
    else:
        workload = (f"n78 100 MHz 4x4 slot, 273 PRB, 64 UEs x 4-5 PRB, 256QAM MCS27, DM-RS symbols 2+11; "
                    f"DL 4 layers, UL {prof['ul_desc']}; LDPC BG1")

    result = {
        "metric": "PDSCH+PUSCH slots/sec (100MHz 4x4) + LDPC info-bits/s at 1/2/4/8 GPU",
        "value": value,
        "unit": "slots/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / steps,
        "higher_is_better": True,
        "scaling": "weak" if args.shard == "cells" else "strong",
        "vs_baseline": None,
        "dtype": "int8/bf16/f32",
        "data": ("synthetic: random TB payloads; PUSCH input = " +
                 ("Gaussian noise samples (no TB ever valid: all LDPC iterations)" if args.worst_case else
                  f"UL TBs through a GPU UE transmitter (same encoder / DM-RS / modulator), a random unitary 4x4 "
                  f"channel and a CFO within +-{CFO_HZ_MAX:g} Hz per UE, AWGN at {args.snr_db:g} dB SNR, "
                  f"OFDM-modulated")),
        "config": {"workload": workload,
                   "profile": args.profile,
                   "workload_kind": args.workload,
                   "dl_chain": "PDSCH encoder -> PDSCH DM-RS -> PDSCH modulator -> OFDM modulator (4 ports)",
                   "ul_chain": "OFDM demodulator (4 ports) -> DM-RS channel estimator (filter, average, CFO "
                               "compensation, TA) -> PUSCH demodulator -> PUSCH decoder",
                   "channel_estimate_layout": "compact (one row per allocation, CFO rotation in the demodulator)"
                                              if ul.estimate_layout == srsgpu.CE_COMPACT else "per symbol",
                   "leg_streams": "one stream" if args.serial_legs else "DL and UL on concurrent streams",
                   "launch": ("two captured HIP graphs per step and input set (DL leg, UL leg), each on its own "
                              "stream" if leg_graphs else "one captured HIP graph per step and input set")
                             if args.graph else "eager launches",
                   "pipelining": (f"up to {K} steps in flight: each input set's step runs on its own stream"
                                  if args.pipeline else "steps serialised on one stream"),
                   "slots_per_step": slots_per_step,
                   "dl_slots_per_step": S_dl, "ul_slots_per_step": S_ul,
                   "input_sets": K,
                   "warmup_steps_run": n_warm,  # max(--warmup, input sets), eager and again after the graph capture
                   "working_set_mb": K * set_bytes / 2 ** 20,
                   "timed_region_s": elapsed,
                   "steps_requested": args.steps,
                   "codeblocks_per_step": {"dl": int(sum(sum(s.nof_segments for s in c.segs) * c.nof_slots
                                                     for c in dl_cells)),
                                           "ul": int(sum(s.nof_segments for s in ul_segs) * S_ul)},
                   "ldpc_max_iterations": args.iterations, "ldpc_early_stop": True,
                   "decoder_arithmetic": "avx2/avx512 (SIMD) variant, bit-exact",
                   "ofdm": "4096-point DFT, 122.88 Msps, normal CP",
                   "parallelism": (f"dp{world}: each GPU processes its own cells' slots" if args.shard == "cells" else
                                   f"ue-shard{world}: the 64 UEs of each slot split across {world} GPUs; OFDM of the "
                                   f"cell on rank 0, resource grids exchanged by subcarrier band over RCCL (UL scatter "
                                   f"after the OFDM demodulation, DL gather before the OFDM modulation: "
                                   f"{2 * sum(gx_ul.bytes_per_rank[1:]) / 2 ** 20:.1f} MB per step)"
                                   if shard_x else "ue-shard1") + (
                                      "; decoded UL TBs + CRC flags gathered to the FAPI rank over RCCL every step"
                                      if tb_gather is not None else "")},
        "tb_gather": None if tb_gather is None else {
            "backend": dist.get_backend(), "world": world, "per_input_set": True,
            "in_graph": bool(args.graph_collectives and sets[0].graph_ul is not None),
            "bytes_per_rank_per_step": int(tb_gather.max_bytes + tb_gather.max_tbs)},
        "ldpc_info_bits_per_s": info_bits_slot * S_ul * step_rate,
        "tb_bits_per_s": {"dl": tbs_bits_dl_step * step_rate, "ul": tbs_bits_ul_step * step_rate},
        "realtime_cells_per_gpu": value / SLOT_RATE_30KHZ / world,
        "pusch_tb_success_rate": tb_success,
        "ldpc_avg_iterations": avg_iters,
        "operating_points": points,
        "stage_ms_per_step": stage,  # from an untimed eager pass with per-stage events
        "stage_algorithmic_gbps": stage_gbps,
        "stage_algorithmic_bytes": stage_bytes,  # per step = per launch of each stage's kernel
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": dec_kernel,
                     "kernel_ms_per_launch": dec_ms, "algorithmic_bytes_per_launch": dec_bytes,
                     "workload_key": wl_key,
                     "note": "algorithmic bytes per launch / decoder-stage HIP-event time on the launch stream (an "
                             "eager pass right after the timed loop); the LDPC decoder is VALU-issue/latency-bound, "
                             "not HBM-bound (DESIGN.md)"},
        "roofline_valu": valu,
        "cpu_baseline": None,
    }
    if skip:
        result["INVALID_timing_experiment_skipped_stages"] = skip
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        n_dl, n_ul = len(dl_segs), len(ul_segs)
        tb_host = st0.dl_tbs[: sum(dl.tb_bytes[:n_dl])].cpu().numpy()
        cw_host = (dl.d_cw.cpu().numpy(), dl.cw_offsets[:n_dl])
        samples_host = st0.samples[: 2 * 4 * 61440].cpu().numpy()
        base, ref_llr, ref_iters = cpu_baseline(
            dl_ues, dl_segs, ul_ues, ul_segs, tb_host, cw_host, samples_host, args.iterations, args.cpu_seconds,
            host_cores(), tdd=(slotlib.TDD_DL_SLOTS + 1, slotlib.TDD_UL_SLOTS) if testmode else None,
            ul_slot_index=ul_cell.slot_index(0))
        result["cpu_baseline"] = base
        if ref_llr is not None and args.profile == "ref":  # the reference shim runs UL slot 0
            # The GPU's UL LLRs of slot 0 against the reference's on the same received samples, and both decoders'
            # codeblock CRC outcomes on slot 0 (each on its own LLRs).
            whole(st0)
            torch.cuda.synchronize()
            got = ul.d_llrs[: sum(s.cw_length for s in ul_segs)].cpu().numpy().astype(np.int16)
            d = np.abs(got - ref_llr.astype(np.int16))
            n_cb0 = sum(s.nof_segments for s in ul_segs)
            gpu_cb_ok = ul.d_crc[:n_cb0].cpu().numpy().astype(bool)
            result["ul_llr_parity_vs_reference"] = {
                "slot": ul_cell.slot_index(0), "llrs": int(d.size), "equal": float(np.mean(d == 0)),
                "within_one_step": float(np.mean(d <= 1)), "max_diff": int(d.max()),
                "codeblocks": n_cb0, "gpu_cb_crc_ok": float(gpu_cb_ok.mean()),
                "reference_cb_crc_ok": float(np.mean(ref_iters >= 0)),
                "cb_outcome_agreement": float(np.mean(gpu_cb_ok == (ref_iters >= 0))),
                "over_one_step": int(np.sum(d > 1)),
                "reference_build_spread": reference_build_spread(ul_ues, samples_host, ul_cell.slot_index(0),
                                                                 ref_llr)}
    # Release the working sets (graphs first) before another workload is measured in the same process.
    for st in sets:
        st.graph = st.graph_back = st.graph_ul = None
    del sets
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return result


EXTRA_WORKLOADS = (
    # The metric's literal 100 MHz 4x4 UL: 4-layer PUSCH per UE + 4x4 MMSE (extension), quoted at 35 dB (four MCS 27
    # layers do not decode at 26 dB).
    ("mimo4_35dB", dict(profile="mimo4", workload="multi_ue", snr_db=35.0)),
    # configs[4]: du_low test mode, continuous max-TBS TDD slots; 30 dB (every 1.18 Mbit TB decodes).
    ("testmode_30dB", dict(profile="ref", workload="testmode", snr_db=30.0)),
)


def summary(r):
    """The fields of a secondary workload kept in the headline line."""
    keys = ("value", "unit", "steps", "ms_per_step", "config", "ldpc_info_bits_per_s", "tb_bits_per_s",
            "realtime_cells_per_gpu", "pusch_tb_success_rate", "ldpc_avg_iterations", "stage_ms_per_step",
            "roofline", "roofline_valu", "cpu_baseline", "ul_llr_parity_vs_reference", "data")
    return {k: r[k] for k in keys if k in r}


def main():
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1 or (args.tb_gather == "always" and "MASTER_ADDR" in os.environ):
        dist.init_process_group("nccl", device_id=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    env = {"ctx": srsgpu.Context(local_rank), "dev": dev, "gen": gen, "world": world, "rank": rank}
    result = measure(args, env)
    if args.extra_workloads and not args.worst_case:
        result["workloads"] = {}
        for name, over in EXTRA_WORKLOADS:
            if over["workload"] == "testmode" and args.shard == "ues" and world > 1:
                continue
            a = argparse.Namespace(**vars(args))
            for k, v in over.items():
                setattr(a, k, v)
            a.extra_points = False
            a.steps = min(args.steps, 400)
            a.min_time = args.min_time / 2
            a.cpu_seconds = args.cpu_seconds / 2
            a.no_cpu_baseline = args.no_cpu_baseline or a.profile != "ref"  # the reference estimates one layer
            result["workloads"][name] = summary(measure(a, env))
    if rank == 0:
        print(json.dumps(result))
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
