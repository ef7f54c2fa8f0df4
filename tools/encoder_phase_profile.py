#!/usr/bin/env python3
"""Phase breakdown of the packed PDSCH encoder kernel on the bench's DL workload (instrumented build).

Build the instrumented library first (next to, not over, the product library):
    SRSGPU_OUT_DIR=srsran-5g_amd/lib_prof SRSGPU_EXTRA_FLAGS=-DENC_PROFILE bash srsran-5g_amd/build.sh
then on the GPU:
    SRSGPU_LIB=srsran-5g_amd/lib_prof/libsrsgpu_phy.so python tools/encoder_phase_profile.py

Each codeblock's workgroup stamps s_memtime at: start (0), after the inline TB CRC (1), after the message bytes (2),
after the CB CRC (3), after the message words (4), after the core rows (5), after p0..p3 (6), after the extension
rows (7), after rate matching (8); s_memrealtime (100 MHz) at start / end (9 / 10).
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "srsran-5g_amd"))

import torch  # noqa: E402

import srsgpu  # noqa: E402
from srsgpu import sch  # noqa: E402

SLOTS = 16
PHASES = ["tb_crc", "msg_bytes", "cb_crc", "msg_words", "core_rows", "core_parity", "ext_rows", "rate_match"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", type=int, default=32)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234)
    ctx = srsgpu.Context(0)
    lib = srsgpu.load_library()
    if not hasattr(lib, "srsgpu_debug_encoder_profile"):
        raise SystemExit("not an instrumented build (set SRSGPU_LIB to the ENC_PROFILE library)")
    ues = sch.slot_100mhz_4x4(nof_layers=4, nof_dmrs_symbols=2)
    segs = [u.segmentation() for u in ues]
    S = args.slots
    tb_bytes = [s.tbs // 8 for s in segs] * S
    cfgs = [srsgpu.PdschTransportBlock(s.base_graph, 0, u.qm, u.nof_layers, u.nof_ch_symbols)
            for u, s in zip(ues, segs)] * S
    arr, tb_total, cw_total, cw_offsets = srsgpu.make_pdsch_configs(tb_bytes, cfgs)
    tbs = torch.randint(0, 256, (tb_total,), generator=gen, device=dev, dtype=torch.uint8)
    cw = torch.zeros(cw_total, dtype=torch.uint8, device=dev)
    enc = srsgpu.PdschEncoderPlan(ctx, arr)
    for _ in range(3):
        enc.execute(tbs, cw)
    torch.cuda.synchronize()
    ncb = sum(s.nof_segments for s in segs) * S
    n = min(ncb, 8192)
    buf = np.zeros(n * SLOTS, dtype=np.uint64)
    lib.srsgpu_debug_encoder_profile.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    assert lib.srsgpu_debug_encoder_profile(buf.ctypes.data, buf.size) == 0
    p = buf.reshape(n, SLOTS).astype(np.int64)
    ok = (p[:, 10] > p[:, 9]) & (p[:, 8] >= p[:, 0])
    p = p[ok]
    res = {"nof_cbs": int(ok.sum())}
    for k, name in enumerate(PHASES):
        res[name + "_cycles"] = float((p[:, k + 1] - p[:, k]).mean())
    res["total_cycles_per_cb"] = float((p[:, 8] - p[:, 0]).mean())
    last_cb = (p[:, 1] - p[:, 0]) > 2 * np.median(p[:, 1] - p[:, 0]) + 100
    res["tb_crc_cycles_on_tb_crc_carriers"] = float((p[last_cb, 1] - p[last_cb, 0]).mean()) if last_cb.any() else 0.0
    res["tb_crc_carriers"] = int(last_cb.sum())
    wall = (p[:, 10] - p[:, 9]) / 100.0
    res["cb_wall_us_avg"] = float(wall.mean())
    res["kernel_span_us"] = float((p[:, 10].max() - p[:, 9].min()) / 100.0)
    res["avg_resident_cbs"] = float(wall.sum() / max(res["kernel_span_us"], 1e-9))
    res["clock_ghz_est"] = float(((p[:, 8] - p[:, 0]) / np.maximum(wall, 1e-3) / 1e3).mean())
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
