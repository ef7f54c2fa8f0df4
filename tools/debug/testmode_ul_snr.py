#!/usr/bin/env python3
"""Diagnostic: UL decoding of the test-mode cell (one 273-PRB UE per UL slot) against SNR, TDD periods and CFO."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "srsran-5g_amd"))
import srsgpu  # noqa: E402
from srsgpu import slot as slotlib  # noqa: E402

ctx = srsgpu.Context(0)
gen = torch.Generator(device="cuda")
gen.manual_seed(3)
for periods in (1, 2):
    _, _, ul_cell = slotlib.tdd_testmode_cells(periods)
    ul = slotlib.UplinkPipeline(ctx, ul_cell, equalizer=srsgpu.EQ_ZF)
    sent = torch.randint(0, 256, (sum(ul.tb_bytes),), generator=gen, device="cuda", dtype=torch.uint8)
    for cfo in (0.0, 300.0):
        for snr in (22.0, 26.0, 30.0, 34.0):
            x = slotlib.synthesize_uplink(ctx, ul_cell, sent, snr_db=snr, seed=99, cfo_hz_max=cfo)
            ul.execute(x, torch.cuda.current_stream())
            torch.cuda.synchronize()
            ok = ul.d_tb_ok.cpu().numpy()
            it = ul.d_iters.cpu().numpy()
            cb_ok = ul.d_crc.cpu().numpy()
            m = ul.d_metrics.cpu().numpy().reshape(-1, srsgpu.CHEST_METRICS)
            print(f"P={periods} cfo={cfo:g} snr={snr:g}: tb_ok {ok.tolist()} cb_ok {cb_ok.mean():.3f} "
                  f"iters {np.where(it > 0, it, 6).mean():.2f} sinr_db {10 * np.log10(m[:, 3]).round(1).tolist()[:8]} "
                  f"ta {m[:4, 4].tolist()} cfo {m[:4, 5].tolist()}", flush=True)
