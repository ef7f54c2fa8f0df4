#!/usr/bin/env python3
"""Phase breakdown of the PUSCH channel estimator kernel (instrumented build), per job.

Build the instrumented library first (next to, not over, the product library):
    SRSGPU_OUT_DIR=srsran-5g_amd/lib_prof SRSGPU_EXTRA_FLAGS=-DCHEST_PROFILE bash srsran-5g_amd/build.sh
then on the GPU:
    SRSGPU_LIB=srsran-5g_amd/lib_prof/libsrsgpu_phy.so python tools/chest_phase_profile.py

Each job's first lane stamps s_memtime after: start (0), sequence staging (1), LSE (2), CFO estimate and
compensation (3), planes (virtual pilots + smoothing) (4), RSRP / noise sums (5), time alignment (6), estimate
writes (7); s_memrealtime (100 MHz) at start / end (10 / 11). Cases: the test-mode 273-PRB UE (one job per rx port,
1024 lanes each) and 16 UEs x 17 PRB.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "srsran-5g_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]

import torch  # noqa: E402

import srsgpu  # noqa: E402
import ul273_cases as U  # noqa: E402

SLOTS = 12
PHASES = ["seq_staging", "lse", "cfo", "planes", "sums", "time_alignment", "estimates"]


def run_case(ctx, lib, name, ests, grid):
    dev = torch.device("cuda", 0)
    nprb = 273
    plan = srsgpu.PuschChannelEstimatorPlan(ctx, srsgpu.make_pusch_chest_configs(ests, [0] * len(ests)), nprb, 4)
    g4 = torch.from_numpy(np.ascontiguousarray(grid).view(np.int32).reshape(-1).copy()).to(dev)
    d_ce = torch.zeros(4 * 4 * 14 * 12 * nprb, dtype=torch.int32, device=dev)
    d_nv = torch.zeros(4 * len(ests), dtype=torch.float32, device=dev)
    for _ in range(5):
        plan.execute(g4, d_ce, d_nv)
    torch.cuda.synchronize()
    njobs = 4 * len(ests)
    buf = np.zeros(4096 * SLOTS, dtype=np.uint64)
    assert lib.srsgpu_debug_chest_profile(buf.ctypes.data_as(srsgpu.ctypes.c_void_p), buf.size) == 0
    st = buf.reshape(4096, SLOTS)[:njobs].astype(np.int64)
    d = np.diff(st[:, :8], axis=1)
    wall_us = (st[:, 11] - st[:, 10]) / 100.0
    ta = {"ta_zero_scatter": float((st[:, 8] - st[:, 5]).mean()), "ta_dft": float((st[:, 9] - st[:, 8]).mean()),
          "ta_corr_argmax": float((st[:, 6] - st[:, 9]).mean())}
    res = {"case": name, "jobs": njobs, "time_alignment_split": ta, "cycles_per_phase_mean": dict(zip(PHASES, d.mean(axis=0).round(1).tolist())),
           "cycles_total_mean": float((st[:, 7] - st[:, 0]).mean()), "job_wall_us_mean": float(wall_us.mean()),
           "job_wall_us_max": float(wall_us.max())}
    print(json.dumps(res), flush=True)
    return res


def main():
    ctx = srsgpu.Context(0)
    lib = srsgpu.load_library()
    if not hasattr(lib, "srsgpu_debug_chest_profile"):
        raise SystemExit("not an instrumented build (set SRSGPU_LIB to the CHEST_PROFILE library)")
    rng = np.random.default_rng(5)
    cfg, _, grid = U.ul273_case(rng, snr_db=26.0)

    def est(rb0, nrb, layout=srsgpu.CE_PER_SYMBOL):
        return srsgpu.PuschChannelEstimation(
            scrambling_id=500, n_scid=0, dmrs_type=1, nof_tx_layers=1, nof_rx_ports=4, start_symbol=0, nof_symbols=14,
            dmrs_symbol_mask=U.DMRS_MASK, rb_start=rb0, nof_rb=nrb, slot_index=cfg["slot"], scaling=U.DMRS_BETA,
            fd_smoothing=2, td_strategy=0, compensate_cfo=1, estimate_layout=layout)

    bench_ues, rb = [], 0
    for i in range(64):  # the bench's slot: 64 UEs x 4-5 PRB, compact layout
        nrb = 5 if i < 17 else 4
        bench_ues.append(est(rb, nrb, srsgpu.CE_COMPACT))
        rb += nrb
    out = [run_case(ctx, lib, "273 PRB, 1 UE, 4 ports", [est(0, 273)], grid),
           run_case(ctx, lib, "273 PRB, 1 UE, 4 ports, compact", [est(0, 273, srsgpu.CE_COMPACT)], grid),
           run_case(ctx, lib, "16 UEs x 17 PRB, 4 ports", [est(17 * i, 17) for i in range(16)], grid),
           run_case(ctx, lib, "64 UEs x 4-5 PRB, 4 ports, compact (bench slot)", bench_ues, grid)]
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "chest_phase_profile.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
